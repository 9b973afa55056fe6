"""Adam on the HIP library (spnerf_adam_step): the training loop's optimizer step.

Reference: main.py:97 builds ``torch.optim.Adam(parameters, lr=args.lr, weight_decay=0)``
(default betas / eps).  Same update as torch's single-tensor Adam, one launch for the whole parameter list
instead of torch's fused multi-tensor kernel (~100 µs per C2 step for 2.7 M parameters).
Parameters must be fp32 CUDA tensors; ``state_dict`` / ``load_state_dict`` follow torch's Adam
layout (``step``, ``exp_avg``, ``exp_avg_sq`` per parameter).
"""
import ctypes

import torch

from . import _lib


class Adam(torch.optim.Optimizer):
    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8):
        if lr < 0.0 or eps <= 0.0 or not (0.0 <= betas[0] < 1.0 and 0.0 <= betas[1] < 1.0):
            raise ValueError(f"bad Adam hyper-parameters lr={lr} betas={betas} eps={eps}")
        super().__init__(params, dict(lr=lr, betas=tuple(betas), eps=eps))

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            ps = [p for p in group["params"] if p.grad is not None]
            if not ps:
                continue
            by_step = {}
            for p in ps:
                if p.dtype != torch.float32 or not p.is_cuda or not p.is_contiguous() or p.grad.is_sparse:
                    raise _lib.SpnerfError("spnerf_amd.optim.Adam: parameters must be contiguous fp32 CUDA tensors")
                st = self.state[p]
                if not st:
                    st["step"] = torch.tensor(0.0)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["step"] += 1
                by_step.setdefault(int(st["step"].item()), []).append(p)
            b1, b2 = group["betas"]
            for step, plist in by_step.items():
                grads = [p.grad if p.grad.is_contiguous() else p.grad.contiguous() for p in plist]
                n = len(plist)
                arr = lambda ts: (ctypes.c_void_p * n)(*[t.data_ptr() for t in ts])
                numel = (ctypes.c_int64 * n)(*[p.numel() for p in plist])
                _lib.check(_lib.lib().spnerf_adam_step(
                    n, arr(plist), arr(grads), arr([self.state[p]["exp_avg"] for p in plist]),
                    arr([self.state[p]["exp_avg_sq"] for p in plist]), numel, group["lr"], b1, b2, group["eps"],
                    step, _lib.stream_of(plist[0])), "adam_step")
        return loss
