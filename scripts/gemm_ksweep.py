"""Split a GEMM's time into its per-K-step main loop and its fixed per-tile part
(prologue + epilogue stores) without instrumenting the kernel: time y = x w^T (bf16) at
fixed M x N over a K sweep and fit t(K) = t0 + K * c.  c / (flop per K) gives the main
loop's MFMA rate, t0 the prologue + epilogue cost per launch.

python scripts/gemm_ksweep.py [--rows 1605632] [--n 1152,384,1536] [--iters 5]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ssl-vit-video-analytics_amd")]

import torch  # noqa: E402

from ssl_mae_amd import kernels as K  # noqa: E402


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=256 * 6272)
    ap.add_argument("--n", default="1152,384,1536")
    ap.add_argument("--ks", default="64,128,192,256,384,512,768,1536")
    ap.add_argument("--iters", type=int, default=5)
    args = ap.parse_args()
    M = args.rows
    ks = [int(v) for v in args.ks.split(",")]
    for N in (int(v) for v in args.n.split(",")):
        pts = []
        for Kd in ks:
            x = torch.randn(M, Kd, device="cuda").to(torch.bfloat16)
            w = torch.randn(N, Kd, device="cuda").to(torch.bfloat16)
            t = timeit(lambda: K.linear(x, w), args.iters)
            f = 2.0 * M * N * Kd
            by = (M * Kd + N * Kd + M * N) * 2
            pts.append((Kd, t))
            print(f"N={N} K={Kd:5d}: {t:8.3f} ms  {f / t / 1e9:7.1f} TF/s  {by / t / 1e6:7.1f} GB/s", flush=True)
            del x, w
            torch.cuda.empty_cache()
        n = len(pts)
        mk = sum(k for k, _ in pts) / n
        mt = sum(t for _, t in pts) / n
        c = sum((k - mk) * (t - mt) for k, t in pts) / sum((k - mk) ** 2 for k, _ in pts)
        t0 = mt - c * mk
        rate = 2.0 * M * N / (c * 1e-3) / 1e12
        print(f"N={N}: fit t(K) = {t0:.3f} ms + K x {c * 1e3:.3f} us  -> main loop {rate:.0f} TF/s "
              f"({rate / 2500:.2f} of peak), fixed part {t0:.3f} ms (output {M * N * 2 / 1e9:.2f} GB "
              f"= {M * N * 2 / (t0 * 1e-3) / 1e12:.2f} TB/s if all stores)", flush=True)


if __name__ == "__main__":
    main()
