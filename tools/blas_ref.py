"""Library reference for the MLP's GEMM shapes: torch.matmul (hipBLASLt / rocBLAS on ROCm) in bf16
with fp32 accumulation, timed by HIP events.  Plain GEMMs (no epilogue, no split-K reduction
choices of ours): what the vendor library reaches on the same shapes on the same chip."""
import sys
import torch

P = int(sys.argv[1]) if len(sys.argv) > 1 else 524288
dev = "cuda:0"


def t(f, iters=20):
    for _ in range(3):
        f()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(iters):
        f()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3


for N, K in ((512, 512), (768, 512), (256, 256)):
    A = torch.randn(P, K, device=dev, dtype=torch.bfloat16)
    W = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.05
    us = t(lambda: A @ W.t())
    print(f"NT  C[{P}x{N}] = A[{P}x{K}] W^T: {us:8.1f} us  {2.0 * P * N * K / us * 1e-6:7.1f} TF/s  "
          f"{(P * K + P * N) * 2 / us * 1e-3:5.2f} TB/s", flush=True)
for N, K in ((512, 512), (768, 512), (256, 256)):
    H = torch.randn(P, N, device=dev, dtype=torch.bfloat16)
    dZ = torch.randn(P, K, device=dev, dtype=torch.bfloat16)
    us = t(lambda: H.t() @ dZ)
    usf = t(lambda: torch.matmul(H.t(), dZ, out=None).float())
    print(f"TN  dW[{N}x{K}] = H^T dZ over {P} points: {us:8.1f} us  {2.0 * P * N * K / us * 1e-6:7.1f} TF/s  "
          f"{(P * K + P * N) * 2 / us * 1e-3:5.2f} TB/s", flush=True)
