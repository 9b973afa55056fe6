"""HIP-graph replay of a training step (bench.py --graph) vs eager launches — needs an MI355X.

Draws come from a static source (the same tensors every step), so a graph replay and an eager
step see identical inputs and must agree bit for bit: loss and every gradient, also after the
parameters change in place (the captured weight re-pack must pick the new values up)."""
import copy

import pytest
import torch

import golden_util as gu
import spnerf_amd
from spnerf_amd import random_source
from spnerf_amd.losses import DepthLoss, SemanticLoss, SNerfLoss
from test_gpu_parity import DEV, gu_rays

pytestmark = pytest.mark.gpu


class StaticRandom:
    """Same draws every step (pre-drawn on first use, then handed out in call order)."""

    def __init__(self, seed=0):
        self.g = torch.Generator(device=DEV).manual_seed(seed)
        self.cache, self.i = [], 0

    def reset(self):
        self.i = 0

    def _get(self, shape, device):
        if self.i == len(self.cache):
            self.cache.append(torch.rand(tuple(shape), device=device, generator=self.g))
        t = self.cache[self.i]
        assert tuple(t.shape) == tuple(shape)
        self.i += 1
        return t

    def rand(self, shape, device):
        return self._get(shape, device)

    def noise(self, shape, device, noise_std):
        return None if noise_std == 0 else self._get(shape, device)

    def gt_uniform(self, valid_mask, n, device):
        return self._get((valid_mask.shape[0], n), device)


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_graph_replay_matches_eager_step(precision):
    torch.manual_seed(0)
    B = 256
    args = gu.args_of({"args": dict(n_samples=64, n_importance=0, model="sp-nerf", beta=False, guidedsample=True,
                                    sc_lambda=0.1, margin=1e-4, stdscale=1.0, chunk=5120, noise_std=0.0)})
    rays = torch.tensor(gu_rays(B, 3), device=DEV)
    g = torch.Generator().manual_seed(1)
    valid = (torch.rand(B, generator=g) < 0.68).long().to(DEV)
    depths = torch.stack([rays[:, 7] * 0.5, torch.rand(B, generator=g).to(DEV)], 1)
    tstd = torch.full((B,), 0.01, device=DEV)
    sems = torch.randint(0, 3, (B,), generator=g).to(DEV)
    rgbs = torch.rand(B, 3, generator=g).to(DEV)
    m_e = spnerf_amd.SPNeRF(num_sem_classes=3, layers=8, feat=128, mapping=True, sem=True, precision=precision).to(DEV)
    m_g = copy.deepcopy(m_e)
    src = StaticRandom()
    sl, dl, ce = SNerfLoss(lambda_sc=0.1), DepthLoss(1.0, usealldepth=False), SemanticLoss(1.0)

    def fwd_bwd(model):
        src.reset()
        res = spnerf_amd.render_rays({"coarse": model}, args, rays, None, semantics=sems, mode="train", valid_depth=valid,
                                     target_depths=depths, target_std=tstd)
        loss = sl(res, rgbs)[0] + dl(res, depths[:, 0], depths[:, 1], valid, tstd)[0] + ce(res, sems)[0]
        loss.backward()
        return loss

    with random_source(src):
        fwd_bwd(m_e)                     # fills the static draws
        m_e.zero_grad(set_to_none=True)
        m_g.zero_grad(set_to_none=True)
        m_g.invalidate_packed()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            loss_g = fwd_bwd(m_g)
        for it in range(2):
            m_e.zero_grad(set_to_none=True)
            loss_e = fwd_bwd(m_e)
            graph.replay()
            torch.cuda.synchronize()
            assert torch.equal(loss_e, loss_g), (it, float(loss_e), float(loss_g))
            for (n, pe), (_, pg) in zip(m_e.named_parameters(), m_g.named_parameters()):
                assert torch.equal(pe.grad, pg.grad), (it, n)
            with torch.no_grad():        # an in-place update, as the optimizer does
                for pe, pg in zip(m_e.parameters(), m_g.parameters()):
                    pe.mul_(0.97).add_(0.001)
                    pg.mul_(0.97).add_(0.001)


def test_graph_training_matches_eager_training():
    """bench.py's graph mode (captured render+loss+backward, eager fused Adam) trains exactly
    like the eager loop: the same loss at every step."""
    torch.manual_seed(0)
    B = 256
    args = gu.args_of({"args": dict(n_samples=64, n_importance=0, model="sp-nerf", beta=False, guidedsample=True,
                                    sc_lambda=0.1, margin=1e-4, stdscale=1.0, chunk=5120, noise_std=0.0)})
    rays = torch.tensor(gu_rays(B, 5), device=DEV)
    g = torch.Generator().manual_seed(2)
    valid = (torch.rand(B, generator=g) < 0.68).long().to(DEV)
    depths = torch.stack([rays[:, 7] * 0.5, torch.rand(B, generator=g).to(DEV)], 1)
    tstd = torch.full((B,), 0.01, device=DEV)
    sems = torch.randint(0, 3, (B,), generator=g).to(DEV)
    rgbs = torch.rand(B, 3, generator=g).to(DEV)
    m_e = spnerf_amd.SPNeRF(num_sem_classes=3, layers=8, feat=128, mapping=True, sem=True).to(DEV)
    m_g = copy.deepcopy(m_e)
    o_e = torch.optim.Adam(m_e.parameters(), lr=5e-4, fused=True)
    o_g = torch.optim.Adam(m_g.parameters(), lr=5e-4, fused=True)
    src = StaticRandom(3)
    sl, dl, ce = SNerfLoss(lambda_sc=0.1), DepthLoss(1.0, usealldepth=False), SemanticLoss(1.0)

    def fwd_bwd(model):
        src.reset()
        res = spnerf_amd.render_rays({"coarse": model}, args, rays, None, semantics=sems, mode="train", valid_depth=valid,
                                     target_depths=depths, target_std=tstd)
        loss = sl(res, rgbs)[0] + dl(res, depths[:, 0], depths[:, 1], valid, tstd)[0] + ce(res, sems)[0]
        loss.backward()
        return loss

    with random_source(src):
        fwd_bwd(m_e)                        # fill the static draws
        o_e.zero_grad(set_to_none=True)
        m_g.invalidate_packed()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            loss_g = fwd_bwd(m_g)
        le, lg = [], []
        for _ in range(6):
            o_e.zero_grad(set_to_none=True)
            le.append(float(fwd_bwd(m_e)))
            o_e.step()
            graph.replay()
            o_g.step()
            lg.append(float(loss_g))
    assert le == lg, (le, lg)
    assert le[-1] < le[0]


def test_forward_sees_fused_optimizer_updates():
    """torch.optim.Adam(fused=True) mutates parameters without bumping _version; the next
    forward must still use the updated weights (packing is unconditional)."""
    torch.manual_seed(0)
    m = spnerf_amd.SPNeRF(num_sem_classes=3, layers=8, feat=128, mapping=True, sem=True).to(DEV)
    opt = torch.optim.Adam(m.parameters(), lr=1e-2, fused=True)
    xyz = torch.rand(500, 3, device=DEV) * 2 - 1
    lab = torch.randint(0, 3, (500,), device=DEV)
    m(xyz, input_s=lab).sum().backward()
    versions = [p._version for p in m.parameters()]
    opt.step()
    out = m(xyz, input_s=lab)
    fresh = spnerf_amd.SPNeRF(num_sem_classes=3, layers=8, feat=128, mapping=True, sem=True).to(DEV)
    fresh.load_state_dict(m.state_dict())
    ref = fresh(xyz, input_s=lab)
    assert torch.equal(out, ref)
    print("fused Adam bumped versions:", versions != [p._version for p in m.parameters()])


def _allocated(addr: int) -> bool:
    """Is device address ``addr`` inside a block the caching allocator has handed out?"""
    for seg in torch.cuda.memory_snapshot():
        a = seg["address"]
        for blk in seg["blocks"]:
            if a <= addr < a + blk["size"]:
                return blk["state"] == "active_allocated"
            a += blk["size"]
    return False


class _Drop(list):
    """A _graph_packs that forgets what it is given (round 5's code before the fix)."""

    def append(self, x):
        pass


@pytest.mark.parametrize("keep", [True, False], ids=["fixed", "round5"])
@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_pooled_pack_outlives_capture(precision, keep):
    """Round 5's illegal-address fault (bench.py's paired replays), step by step:
    an eager step returns its packed-weight buffer to the model's free list; the capture takes
    that buffer (allocated OUTSIDE the graph's private pool); a SECOND capture follows, whose
    torch.cuda.graph.__enter__ calls torch.cuda.empty_cache(); eager tensors of the buffer's size
    are allocated.  Fixed (the buffer kept with the graph, SPNeRF.release_graph_packs): it stays
    allocated, no eager tensor overlaps it, and replays of the first graph equal eager steps bit
    for bit with the eager tensors untouched.  round5 (the buffer not kept): after the second
    capture its address is no longer allocated — what a replay would have written through; that
    arm never replays."""
    torch.manual_seed(0)
    B = 128
    args = gu.args_of({"args": dict(n_samples=64, n_importance=0, model="sp-nerf", beta=False, guidedsample=True,
                                    sc_lambda=0.1, margin=1e-4, stdscale=1.0, chunk=5120, noise_std=0.0)})
    rays = torch.tensor(gu_rays(B, 7), device=DEV)
    g = torch.Generator().manual_seed(4)
    valid = (torch.rand(B, generator=g) < 0.68).long().to(DEV)
    depths = torch.stack([rays[:, 7] * 0.5, torch.rand(B, generator=g).to(DEV)], 1)
    tstd = torch.full((B,), 0.01, device=DEV)
    sems = torch.randint(0, 3, (B,), generator=g).to(DEV)
    rgbs = torch.rand(B, 3, generator=g).to(DEV)
    m = spnerf_amd.SPNeRF(num_sem_classes=3, layers=8, feat=128, mapping=True, sem=True, precision=precision).to(DEV)
    m_ref = copy.deepcopy(m)
    if not keep:
        m._graph_packs = _Drop()
    src = StaticRandom(5)
    sl, dl, ce = SNerfLoss(lambda_sc=0.1), DepthLoss(1.0, usealldepth=False), SemanticLoss(1.0)

    def fwd_bwd(model):
        src.reset()
        res = spnerf_amd.render_rays({"coarse": model}, args, rays, None, semantics=sems, mode="train", valid_depth=valid,
                                     target_depths=depths, target_std=tstd)
        loss = sl(res, rgbs)[0] + dl(res, depths[:, 0], depths[:, 1], valid, tstd)[0] + ce(res, sems)[0]
        loss.backward()
        return loss

    with random_source(src):
        fwd_bwd(m)                                   # eager: its own pack goes back to the free list
        assert len(m._pack_pool) == 1
        addr, nbytes = m._pack_pool[0].data_ptr(), 4 * m._pack_pool[0].numel()
        m.zero_grad(set_to_none=True)
        g1 = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g1):
            loss_g = fwd_bwd(m)
        assert not m._pack_pool                      # the capture took the pooled buffer
        g2 = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g2):                   # __enter__: synchronize + empty_cache
            fwd_bwd(m)
        torch.cuda.synchronize()
        if not keep:
            assert not _allocated(addr), "the captured pack survived without being kept"
            del g1, g2
            return
        junk = [torch.full((nbytes // 4,), 7.0, device=DEV) for _ in range(4)]
        packs = m.release_graph_packs()
        assert any(p.data_ptr() == addr for p in packs) and _allocated(addr)
        for j in junk:
            assert j.data_ptr() + nbytes <= addr or addr + nbytes <= j.data_ptr()
        for it in range(2):
            m_ref.zero_grad(set_to_none=True)
            loss_e = fwd_bwd(m_ref)
            g1.replay()
            torch.cuda.synchronize()
            assert torch.equal(loss_e, loss_g), (it, float(loss_e), float(loss_g))
            for (n, pe), (_, pg) in zip(m_ref.named_parameters(), m.named_parameters()):
                assert torch.equal(pe.grad, pg.grad), (it, n)
            assert all(bool((j == 7.0).all()) for j in junk)
            with torch.no_grad():
                for pe, pg in zip(m_ref.parameters(), m.parameters()):
                    pe.mul_(0.97).add_(0.001)
                    pg.mul_(0.97).add_(0.001)
        del g1, g2, packs
