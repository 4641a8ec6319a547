"""Weight-gradient GEMMs of the step: v2 tiles vs the 384 x 128 pipelined tile (sm_gemm_tuning
dw384 0 / 1), interleaved rounds in one process; dW compared (own split counts: fp32 grouping differs).

    python scripts/dw384_ab.py [--rounds 5] [--iters 3]
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
    ap.add_argument("--key", default="dw384", help="the 0 / 1 tuning key to A/B (dw384, dw384_notr)")
    a = ap.parse_args()
    B = a.batch
    dev = "cuda"
    M2 = B * 6272
    for name, rows, nout, nin in [("dec/s2 fc2", M2, 384, 1536), ("dec/s2 fc1", M2, 1536, 384),
                                  ("dec/s2 qkv", M2, 1152, 384), ("dec/s2 proj", M2, 384, 384)]:
        dy = torch.randn(rows, nout, device=dev).to(torch.bfloat16)
        x = torch.randn(rows, nin, device=dev).to(torch.bfloat16)
        gw = {0: torch.zeros(nout, nin, device=dev), 1: torch.zeros(nout, nin, device=dev)}
        gb = {0: torch.zeros(nout, device=dev), 1: torch.zeros(nout, device=dev)}
        times = {0: [], 1: []}
        for _ in range(a.rounds):
            for arm in (0, 1):
                prev = K.gemm_tuning(a.key, arm)
                times[arm].append(timeit(lambda: K.linear_dw_bias(dy, x, gw[arm], gb[arm]), a.iters))
                K.gemm_tuning(a.key, prev)
        same = ((gw[0] - gw[1]).abs().max() / gw[0].abs().max()).item()
        med = {k: sorted(v)[len(v) // 2] for k, v in times.items()}
        f = 2.0 * rows * nout * nin
        print(f"dW {name}: rows={rows} nout={nout} nin={nin}  {a.key}=0 {med[0]:7.3f} ms ({f / med[0] / 1e9:6.1f} TF/s) | "
              f"{a.key}=1 {med[1]:7.3f} ms ({f / med[1] / 1e9:6.1f} TF/s, {(med[1] / med[0] - 1) * 100:+.1f} %) | "
              f"dW max rel diff {same:.1e}", flush=True)
        del dy, x
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
