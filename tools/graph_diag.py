"""Diagnostic: which gradients differ between eager steps and HIP-graph replays, and when."""
import copy
import sys

import torch

sys.path.insert(0, "tests")
sys.path.insert(0, ".")
import golden_util as gu  # noqa: E402
import spnerf_amd  # noqa: E402
from spnerf_amd import random_source  # noqa: E402
from spnerf_amd.losses import DepthLoss, SemanticLoss, SNerfLoss  # noqa: E402
from test_gpu_graph import StaticRandom  # noqa: E402
from test_gpu_parity import DEV, gu_rays  # noqa: E402

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
mode = sys.argv[1] if len(sys.argv) > 1 else "update+eager"
m_e = spnerf_amd.SPNeRF(num_sem_classes=3, layers=8, feat=128, mapping=True, sem=True).to(DEV)
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


import spnerf_amd.spnerf as _sp  # noqa: E402
_orig_bwd = _sp._MLP.backward
_log = []


def _bwd(ctx, d_out):
    r = _orig_bwd(ctx, d_out)
    g = [x for x in r[7:] if x is not None]
    base = g[0]
    _log.append(("mlp_grad_flat", base.untyped_storage().data_ptr(), base.untyped_storage().nbytes(),
                 torch.cuda.is_current_stream_capturing()))
    return r


_sp._MLP.backward = staticmethod(_bwd)

with random_source(src):
    fwd_bwd(m_e)
    m_e.zero_grad(set_to_none=True)
    m_g.zero_grad(set_to_none=True)
    m_g.invalidate_packed()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        loss_g = fwd_bwd(m_g)
    m_e.zero_grad(set_to_none=True)
    loss_e = fwd_bwd(m_e)
    ge0 = [p.grad.clone() for p in m_e.parameters()]
    print("during capture:", [x for x in _log if x[3]])
    _log.clear()
    for n, p in m_g.named_parameters():
        st = p.grad.untyped_storage()
        print(f"  m_g.{n:32s} grad ptr {p.grad.data_ptr():#x} storage {st.data_ptr():#x}+{st.nbytes()} view={p.grad._base is not None}")
    for it in range(3):
        if mode in ("update+eager", "eager-only"):
            m_e.zero_grad(set_to_none=True)
            loss_e = fwd_bwd(m_e)
        elif mode == "fwd-nograd":
            src.reset()
            with torch.no_grad():
                spnerf_amd.render_rays({"coarse": m_e}, args, rays, None, semantics=sems, mode="train", valid_depth=valid,
                                       target_depths=depths, target_std=tstd)
        elif mode == "fwd-grad":
            src.reset()
            keep = spnerf_amd.render_rays({"coarse": m_e}, args, rays, None, semantics=sems, mode="train",
                                          valid_depth=valid, target_depths=depths, target_std=tstd)
        elif mode == "alloc":
            junk = [torch.full((1 << 22,), 1e30, device=DEV) for _ in range(64)]
            del junk
        if _log:
            print("  eager backward flat buffers:", [(hex(a), b) for _, a, b, _c in _log])
            _log.clear()
        graph.replay()
        torch.cuda.synchronize()
        bad = []
        for (n, pe), (_, pg) in zip(m_e.named_parameters(), m_g.named_parameters()):
            if not torch.equal(pe.grad, pg.grad):
                d = (pe.grad - pg.grad).abs()
                idx = torch.nonzero(d > 1e-6 * (1 + pe.grad.abs()))
                bad.append((n, tuple(pe.shape), float(d.max()), idx[:4].tolist(), int(idx.shape[0])))
        print(f"[{mode}] iter {it}: loss eager {float(loss_e):.6f} graph {float(loss_g):.6f}; mismatching grads: {len(bad)}")
        for b in bad:
            print("    ", b)
        if "update" in mode:
            with torch.no_grad():
                for pe, pg in zip(m_e.parameters(), m_g.parameters()):
                    pe.mul_(0.97).add_(0.001)
                    pg.mul_(0.97).add_(0.001)
