"""Compare our GEMM kernel against torch.matmul (hipBLASLt) on the step's shapes."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ssl-vit-video-analytics_amd")]
import torch
from ssl_mae_amd import kernels as K


def timeit(fn, iters=5):
    fn(); torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True); e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


# HBM calibration: write-only (fill) and copy of a 4.9 GB bf16 tensor (fc1's output size)
big = torch.empty(1605632 * 1536, dtype=torch.bfloat16, device="cuda")
nb = big.numel() * 2
t = timeit(lambda: big.fill_(1.0))
print(f"fill (write only) {nb / 1e9:.2f} GB: {t:.3f} ms = {nb / t / 1e6:.0f} GB/s", flush=True)
src = torch.empty_like(big)
t = timeit(lambda: big.copy_(src))
print(f"copy {nb / 1e9:.2f} GB each way: {t:.3f} ms = {2 * nb / t / 1e6:.0f} GB/s (read+write)", flush=True)
t = timeit(lambda: src.sum())
print(f"sum (read only) {nb / 1e9:.2f} GB: {t:.3f} ms = {nb / t / 1e6:.0f} GB/s", flush=True)
del big, src
torch.cuda.empty_cache()

for name, M, N, Kd in [("fc1", 1605632, 1536, 384), ("fc2", 1605632, 384, 1536), ("qkv", 1605632, 1152, 384),
                       ("s0exp", 6422528, 384, 96), ("s0proj", 6422528, 96, 384)]:
    x = torch.randn(M, Kd, device="cuda").to(torch.bfloat16)
    w = torch.randn(N, Kd, device="cuda").to(torch.bfloat16)
    dy = torch.randn(M, N, device="cuda").to(torch.bfloat16)
    f = 2.0 * M * N * Kd
    ours_f = timeit(lambda: K.linear(x, w))
    blas_f = timeit(lambda: torch.matmul(x, w.t()))
    ours_dx = timeit(lambda: K.linear_dx(dy, w))
    blas_dx = timeit(lambda: torch.matmul(dy, w))
    sink = torch.zeros(N, Kd, device="cuda")
    ours_dw = timeit(lambda: K.linear_dw(dy, x, sink))
    blas_dw = timeit(lambda: torch.matmul(dy.t(), x.float().to(torch.bfloat16)) if False else torch.matmul(dy.t(), x))
    print(f"{name}: M={M} N={N} K={Kd} | fwd ours {f/ours_f/1e9:6.0f} blas {f/blas_f/1e9:6.0f} TF/s | "
          f"dX ours {f/ours_dx/1e9:6.0f} blas {f/blas_dx/1e9:6.0f} | dW ours {f/ours_dw/1e9:6.0f} blas {f/blas_dw/1e9:6.0f}",
          flush=True)
    del x, w, dy, sink
    torch.cuda.empty_cache()
