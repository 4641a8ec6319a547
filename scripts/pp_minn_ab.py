"""Persistent GEMM form below its N >= 512 rule: the stage-1 / stage-2 Linear shapes with
N = 192 / 384 / 576 (K <= 384), minimum N 512 vs 128 (pp_min_n), interleaved rounds in one
process; outputs compared bitwise (the persistent form is bit-identical to v2).

    python scripts/pp_minn_ab.py [--rounds 5] [--iters 3]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ssl-vit-video-analytics_amd")]

import torch  # noqa: E402

from ssl_mae_amd import kernels as K  # noqa: E402
from kbench import timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--maxk", action="store_true",
                    help="instead: K > 384 shapes, pp_max_k 384 (default) vs 1536 (minimum N 0 for both layouts)")
    ap.add_argument("--dx", action="store_true",
                    help="instead: data-gradient shapes, v2 vs persistent at every K (pp_min_n 0, pp_max_k 1536 "
                         "against pp disabled)")
    ap.add_argument("--arms", default="",
                    help="JSON list of gemm_tuning dicts to compare instead (first = baseline), e.g. "
                         "'[{\"pp_rounds_mid_k\": 2}, {\"pp_rounds_mid_k\": 4}]'")
    a = ap.parse_args()
    B = a.batch
    dev = "cuda"
    M1, M2 = B * 8 * 3136, B * 8 * 784
    # (name, kind, M, N_out, K_red)
    cases = [("s1 proj fwd", "fwd", M1, 192, 192), ("s1 qkv fwd", "fwd", M1, 576, 192),
             ("s1 proj dX", "dx", M1, 192, 192), ("s1 qkv dX", "dx", M1, 192, 576),
             ("s2/dec proj fwd", "fwd", M2, 384, 384), ("s2/dec proj dX", "dx", M2, 384, 384)]
    if a.dx:
        cases = [("s1 proj dX", "dx", M1, 192, 192), ("s2/dec proj dX", "dx", M2, 384, 384),
                 ("dec fc2 dX", "dx", M2, 1536, 384), ("s1 qkv dX", "dx", M1, 192, 576),
                 ("dec qkv dX", "dx", M2, 384, 1152), ("dec fc1 dX", "dx", M2, 384, 1536),
                 ("s0 proj dX (N = 96)", "dx", B * 8 * 12544, 96, 384)]
    if a.maxk:
        cases = [("dec fc2 fwd", "fwd", M2, 384, 1536), ("s1 fc2 fwd", "fwd", M1, 192, 768),
                 ("dec qkv dX", "dx", M2, 384, 1152), ("dec fc1 dX", "dx", M2, 384, 1536),
                 ("s1 fc1 dX", "dx", M1, 192, 768)]
    for name, kind, M, N, Kd in cases:
        x = torch.randn(M, Kd, device=dev).to(torch.bfloat16)
        if kind == "fwd":
            w = (torch.randn(N, Kd, device=dev) * 0.05).to(torch.bfloat16)
            b = torch.randn(N, device=dev)
            fn = lambda: K.linear(x, w, b)  # noqa: E731
        else:   # dx[M][N] = dy[M][Kd] w[Kd][N]
            w = (torch.randn(Kd, N, device=dev) * 0.05).to(torch.bfloat16)
            fn = lambda: K.linear_dx(x, w)  # noqa: E731
        arms = ({"pp_min_n": 512}, {"pp_min_n": 128})
        if a.dx:
            arms = ({"pp": 0}, {"pp": 1, "pp_min_n": 0, "pp_max_k": 1536})
        if a.maxk:
            arms = ({"pp_min_n": 0, "pp_max_k": 384}, {"pp_min_n": 0, "pp_max_k": 1536})
        if a.arms:
            import json
            arms = tuple(json.loads(a.arms))
        times = {i: [] for i in range(len(arms))}
        outs = {}
        for _ in range(a.rounds):
            for arm in range(len(arms)):
                prev = {k: K.gemm_tuning(k, v) for k, v in arms[arm].items()}
                times[arm].append(timeit(fn, a.iters))
                outs[arm] = fn()
                for k, v in prev.items():
                    K.gemm_tuning(k, v)
        same = all(torch.equal(outs[0], outs[i]) for i in outs)
        med = {k: sorted(v)[len(v) // 2] for k, v in times.items()}
        if not a.arms:
            print(f"{name}: M={M} N={N} K={Kd}  v2 rule {med[0]:7.3f} ms | persistent {med[1]:7.3f} ms "
                  f"({(med[1] / med[0] - 1) * 100:+.1f} %) | bit-identical {same}", flush=True)
        else:
            cols = " | ".join(f"{json.dumps(arms[i])} {med[i]:7.3f} ms ({(med[i] / med[0] - 1) * 100:+.1f} %)"
                              for i in range(len(arms)))
            print(f"{name}: M={M} N={N} K={Kd}  {cols} | bit-identical {same}", flush=True)
        del x, w, outs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
