"""Same-process A/B of the forward GEMM kernels (knob 'gemm_dma': register-staged v2 vs
the LDS-DMA ring) at the step's K-major shapes, alternating the variants per repetition.

python scripts/gemm_dma_ab.py [--reps 3] [--iters 5]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ssl-vit-video-analytics_amd")]

import torch  # noqa: E402

from ssl_mae_amd import kernels as K  # noqa: E402
from gemm_ksweep import timeit  # noqa: E402

B = 256
SHAPES = [  # (name, M, N, K, bias, gelu, stats); "dX": dy [M, K] @ w [K, N]; "dXg": + GELU backward
    ("dec qkv fwd", B * 6272, 1152, 384, True, False, False),
    ("dec fc1+gelu fwd", B * 6272, 1536, 384, True, True, False),
    ("dec fc2 fwd", B * 6272, 384, 1536, True, False, False),
    ("dec proj fwd", B * 6272, 384, 384, True, False, False),
    ("s0 expand+stats", B * 8 * 12544, 384, 96, False, False, True),
    ("s1 qkv fwd", B * 8 * 3136, 576, 192, True, False, False),
    ("s1 fc1+gelu", B * 8 * 3136, 768, 192, True, True, False),
    ("dec qkv dX", B * 6272, 384, 1152, False, "dX", False),
    ("dec fc1 dX", B * 6272, 384, 1536, False, "dX", False),
    ("dec fc2 dX+gelu", B * 6272, 1536, 384, False, "dXg", False),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--only", default="")
    ap.add_argument("--variants", default="0,1,2", help="gemm_dma knob values: 0 v2, 1 DMA 3-stage, 2 DMA 6-stage")
    args = ap.parse_args()
    for name, M, N, Kd, bias, gelu, stats in SHAPES:
        if args.only and args.only not in name:
            continue
        x = torch.randn(M, Kd, device="cuda").to(torch.bfloat16)
        w = (torch.randn(N, Kd, device="cuda") * 0.05).to(torch.bfloat16)
        b = torch.randn(N, device="cuda") if bias else None
        if gelu in ("dX", "dXg"):            # dx [M, N] = dy [M, K] @ wt [K, N]
            wt = (torch.randn(Kd, N, device="cuda") * 0.05).to(torch.bfloat16)
            if gelu == "dX":
                fn = lambda: K.linear_dx(x, wt)  # noqa: E731
            else:
                pre = torch.randn(M, N, device="cuda").to(torch.bfloat16)
                fn = lambda: K.linear_dx_gelu(x, wt, pre, 0.1, 5)  # noqa: E731
        elif stats:
            fn = lambda: K.linear_bn_stats(x, w)  # noqa: E731
        else:
            fn = lambda: K.linear(x, w, b, gelu=gelu)  # noqa: E731
        vs = [int(v) for v in args.variants.split(",")]
        t = {v: [] for v in vs}
        outs = {}
        for _ in range(args.reps):
            for v in vs:
                K.set_tuning("gemm_dma", v)
                t[v].append(timeit(fn, args.iters))
                o = fn()
                outs[v] = o[0] if isinstance(o, tuple) else o
        K.set_tuning("gemm_dma", 0)
        same = all(torch.equal(outs[vs[0]], outs[v]) for v in vs)
        f = 2.0 * M * N * Kd
        t0 = min(t[vs[0]])
        cols = " | ".join(f"knob {v}: {min(t[v]):7.3f} ms ({f / min(t[v]) / 1e9:5.0f} TF/s, {t0 / min(t[v]):4.2f}x)"
                          for v in vs)
        print(f"{name:18s} M={M} N={N} K={Kd}: {cols}  bit-identical {same}", flush=True)
        del x, w, b, outs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
