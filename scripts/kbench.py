"""Kernel micro-benchmarks at the bench shapes (B=256, T=8, 224^2).

python scripts/kbench.py attn [--drop 0.1] [--iters 5]   # decoder (d=64) + encoder (d=32) attention
python scripts/kbench.py gemm                              # the main GEMM shapes
Prints per-kernel-group average ms and TFLOP/s measured with HIP events.
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


def attn(args):
    cases = [("dec d64", args.batch, 6 * 1, 8 * 784, 64, args.drop),
             ("enc1 d32", args.batch * 8, 6, 3136, 32, 0.0),
             ("enc2 d32", args.batch * 8, 12, 784, 32, 0.0)]
    for name, N, H, L, D, p in cases:
        if args.only and args.only not in name:
            continue
        qkv = (torch.randn(N * L, 3 * H * D, device="cuda") * 0.5).to(torch.bfloat16)
        do = torch.randn(N * L, H * D, device="cuda").to(torch.bfloat16)
        o, lse = K.attn_fwd(qkv, N, L, H, D, p, 7)
        f = 4.0 * N * H * L * L * D
        t_f = timeit(lambda: K.attn_fwd(qkv, N, L, H, D, p, 7), args.iters)
        shapes = [int(v) for v in args.bwd_shapes.split(",")] if args.bwd_shapes else [None]
        times = {sh: [] for sh in shapes}
        for _ in range(args.rounds):            # interleaved rounds, one process (guide rule 24)
            for sh in shapes:
                prev = K.attn_tuning(D, sh) if sh else None
                times[sh].append(timeit(lambda: K.attn_bwd(qkv, o, do, lse, N, L, H, D, p, 7), args.iters))
                if sh:
                    K.attn_tuning(D, prev)
        for sh in shapes:
            ts = sorted(times[sh])
            t_b = ts[len(ts) // 2]
            print(f"{name}: N={N} H={H} L={L} D={D} p={p}  fwd {t_f:8.2f} ms {f / t_f / 1e9:7.1f} TF/s | "
                  f"bwd[{sh or 'default'}] median {t_b:8.2f} ms min {ts[0]:8.2f} ms {2 * f / t_b / 1e9:7.1f} TF/s "
                  f"(algorithmic 8BHL^2D)", flush=True)
        del qkv, do, o, lse
        torch.cuda.empty_cache()


def gemm(args):
    B = args.batch
    cases = [  # (name, M, N, K)
        ("dec fc1 fwd", B * 6272, 1536, 384), ("dec fc2 fwd", B * 6272, 384, 1536),
        ("dec qkv fwd", B * 6272, 1152, 384), ("s0 expand fwd", B * 8 * 12544, 384, 96),
        ("s0 proj fwd", B * 8 * 12544, 96, 384), ("s2 fc1 fwd", B * 8 * 784, 1536, 384),
        ("dec proj fwd", B * 6272, 384, 384), ("s1 qkv fwd", B * 8 * 3136, 576, 192)]
    # --mf 32,16: the K loop's MFMA shape A/B (gemm_tuning mf16_min_k: 16 -> every K-major-A
    # v2 GEMM on 16x16x32, 32 -> none), interleaved rounds in one process
    mfs = [int(v) for v in args.mf.split(",")] if args.mf else [None]
    for name, M, N, Kd in cases:
        if args.only and args.only not in name:
            continue
        x = torch.randn(M, Kd, device="cuda").to(torch.bfloat16)
        w = torch.randn(N, Kd, device="cuda").to(torch.bfloat16)
        b = torch.randn(N, device="cuda")
        f = 2.0 * M * N * Kd
        dy = torch.randn(M, N, device="cuda").to(torch.bfloat16)
        sink = torch.zeros(N, Kd, device="cuda")
        ops = {"fwd": lambda: K.linear(x, w, b), "dX": lambda: K.linear_dx(dy, w),
               "dW": lambda: K.linear_dw(dy, x, sink)}
        times = {(mf, o): [] for mf in mfs for o in ops}
        for _ in range(args.rounds):
            for mf in mfs:
                prev = K.gemm_tuning("mf16_min_k", 0 if mf == 16 else 1 << 30) if mf else None
                for o, fn in ops.items():
                    times[(mf, o)].append(timeit(fn, args.iters))
                if mf:
                    K.gemm_tuning("mf16_min_k", prev)
        for mf in mfs:
            med = {o: sorted(times[(mf, o)])[len(times[(mf, o)]) // 2] for o in ops}
            print(f"{name} [mf {mf or 'default'}]: M={M} N={N} K={Kd}  fwd {med['fwd']:7.3f} ms "
                  f"{f / med['fwd'] / 1e9:7.1f} TF/s | dX {med['dX']:7.3f} ms {f / med['dX'] / 1e9:7.1f} | "
                  f"dW {med['dW']:7.3f} ms {f / med['dW'] / 1e9:7.1f}", flush=True)
        del x, w, dy, sink
        torch.cuda.empty_cache()


def bnstats(args):
    """Linear + output BatchNorm statistics (linear_bn_stats: the MBConv expand convs) against
    the plain linear of the same shape: the statistics epilogue's cost."""
    B = args.batch
    for name, M, N, Kd in [("s0 expand+stats", B * 8 * 12544, 384, 96), ("s1 expand+stats", B * 8 * 3136, 768, 192)]:
        x = torch.randn(M, Kd, device="cuda").to(torch.bfloat16)
        w = torch.randn(N, Kd, device="cuda").to(torch.bfloat16)
        t0 = timeit(lambda: K.linear(x, w), args.iters)
        t1 = timeit(lambda: K.linear_bn_stats(x, w), args.iters)
        print(f"{name}: M={M} N={N} K={Kd}  linear {t0:7.3f} ms | linear_bn_stats {t1:7.3f} ms "
              f"(statistics +{t1 - t0:6.3f} ms)", flush=True)
        del x, w
        torch.cuda.empty_cache()


def dw(args):
    """Every weight-gradient GEMM shape of the step: dW[nout][nin] = dy^T x (+ db)."""
    B = args.batch
    cases = [("dec/s2 fc2", B * 6272, 384, 1536), ("dec/s2 fc1", B * 6272, 1536, 384),
             ("dec/s2 qkv", B * 6272, 1152, 384), ("dec/s2 proj", B * 6272, 384, 384),
             ("s1 fc1", B * 8 * 3136, 768, 192), ("s1 fc2", B * 8 * 3136, 192, 768),
             ("s1 qkv", B * 8 * 3136, 576, 192), ("s1 proj", B * 8 * 3136, 192, 192),
             ("s0 expand", B * 8 * 12544, 384, 96), ("s0 proj", B * 8 * 12544, 96, 384)]
    for name, M, nout, nin in cases:
        if args.only and args.only not in name:
            continue
        dy = torch.randn(M, nout, device="cuda").to(torch.bfloat16)
        x = torch.randn(M, nin, device="cuda").to(torch.bfloat16)
        gw = torch.zeros(nout, nin, device="cuda")
        gb = torch.zeros(nout, device="cuda")
        f = 2.0 * M * nout * nin
        t = timeit(lambda: K.linear_dw_bias(dy, x, gw, gb), args.iters)
        print(f"dW {name}: rows={M} nout={nout} nin={nin}  {t:7.3f} ms {f / t / 1e9:7.1f} TF/s", flush=True)
        del dy, x, gw, gb
        torch.cuda.empty_cache()


def dwx(args):
    """fc2 weight gradients of dropout(GELU(pre)) (linear_dw_bias gelu=) against the gelu
    recompute kernel + plain weight gradient; outputs compared bitwise."""
    B = args.batch
    dev = "cuda"
    for name, M, H, nout, p in [("dec fc2", B * 6272, 1536, 384, 0.1), ("s2 fc2", B * 8 * 784, 1536, 384, 0.0),
                                ("s1 fc2", B * 8 * 3136, 768, 192, 0.0)]:
        pre = torch.randn(M, H, device=dev).to(torch.bfloat16)
        dy = (torch.randn(M, nout, device=dev) * 0.1).to(torch.bfloat16)
        gw1, gb1 = torch.zeros(nout, H, device=dev), torch.zeros(nout, device=dev)
        gw2, gb2 = torch.zeros(nout, H, device=dev), torch.zeros(nout, device=dev)
        K.linear_dw_bias(dy, K.gelu(pre, p, 77), gw1, gb1)
        K.linear_dw_bias(dy, pre, gw2, gb2, gelu=(p, 77))
        same = torch.equal(gw1, gw2) and torch.equal(gb1, gb2)
        t0 = timeit(lambda: K.linear_dw_bias(dy, K.gelu(pre, p, 77), gw1, gb1), args.iters)
        t1 = timeit(lambda: K.linear_dw_bias(dy, pre, gw2, gb2, gelu=(p, 77)), args.iters)
        print(f"{name}: rows={M} dW[{nout}][{H}] p={p}  gelu kernel + dW {t0:7.3f} ms | dW(gelu=) {t1:7.3f} ms | "
              f"bit-identical {same}", flush=True)
        del pre, dy
        torch.cuda.empty_cache()


def dxgelu(args):
    """fc2 data gradient through dropout(GELU(pre)) with the h side output (linear_dx_gelu):
    persistent form (gemm_bf16_pp IMP 9) against one tile per block (v2), interleaved rounds;
    outputs compared bitwise."""
    B = args.batch
    dev = "cuda"
    for name, M, N, H, p in [("dec fc2", B * 6272, 384, 1536, 0.1), ("s2 fc2", B * 8 * 784, 384, 1536, 0.0),
                             ("s1 fc2", B * 8 * 3136, 192, 768, 0.0), ("s1 fc2 (no h)", B * 8 * 3136, 192, 768, 0.0)]:
        if args.only and args.only not in name:
            continue
        pre = torch.randn(M, H, device=dev).to(torch.bfloat16)
        dy = (torch.randn(M, N, device=dev) * 0.1).to(torch.bfloat16)
        w = (torch.randn(N, H, device=dev) * 0.05).to(torch.bfloat16)
        out = {}
        times = {0: [], 1: []}
        for _ in range(args.rounds):
            for pp in (0, 1):
                prev = K.gemm_persistent(pp)
                if name.endswith("(no h)"):
                    times[pp].append(timeit(lambda: K.linear_dx(dy, w, gelu_pre=pre, drop_p=p, seed=77), args.iters))
                    out[pp] = (K.linear_dx(dy, w, gelu_pre=pre, drop_p=p, seed=77), pre)
                else:
                    times[pp].append(timeit(lambda: K.linear_dx_gelu(dy, w, pre, p, 77), args.iters))
                    out[pp] = K.linear_dx_gelu(dy, w, pre, p, 77)
                K.gemm_persistent(prev)
        same = torch.equal(out[0][0], out[1][0]) and torch.equal(out[0][1], out[1][1])
        med = {k: sorted(v)[len(v) // 2] for k, v in times.items()}
        gb = (M * N + 3 * M * H) * 2 / 1e9
        print(f"{name}: M={M} N={N} H={H} p={p}  v2 {med[0]:7.3f} ms | persistent {med[1]:7.3f} ms "
              f"({gb / med[1]:5.2f} TB/s algorithmic) | bit-identical {same}", flush=True)
        del pre, dy, w, out
        torch.cuda.empty_cache()


def dwse(args):
    """MBConv projection weight gradient over the SE output: se_scale + linear_dw against
    linear_dw_se (h3 formed in the GEMM's operand loads); outputs compared bitwise."""
    B = args.batch
    dev = "cuda"
    for name, Fn, HW, N, C in [("s0 proj", B * 8, 12544, 96, 384), ("s1 down proj", B * 8, 3136, 192, 384)]:
        M = Fn * HW
        a2 = (torch.randn(M, C, device=dev) * 2).to(torch.bfloat16)
        dy = (torch.randn(M, N, device=dev) * 0.1).to(torch.bfloat16)
        act = (torch.zeros(C, device=dev), torch.ones(C, device=dev), torch.ones(C, device=dev),
               torch.zeros(C, device=dev), True)
        gate = torch.rand(Fn, C, device=dev)
        g1, g2 = torch.zeros(N, C, device=dev), torch.zeros(N, C, device=dev)

        def unfused():
            K.linear_dw(dy, K.se_scale(a2, gate, Fn, HW, C, act=act), g1, accumulate=False)
        unfused()
        K.linear_dw_se(dy, a2, act, gate, HW, g2, accumulate=False)
        same = torch.equal(g1, g2)
        t0 = timeit(unfused, args.iters)
        t1 = timeit(lambda: K.linear_dw_se(dy, a2, act, gate, HW, g2, accumulate=False), args.iters)
        print(f"{name}: rows={M} dW[{N}][{C}]  se_scale + dW {t0:7.3f} ms | dW(se operand) {t1:7.3f} ms | "
              f"bit-identical {same}", flush=True)
        if HW % 128 == 0:   # forward: se_fwd's h3 + linear against linear_se
            w = (torch.randn(N, C, device=dev) * 0.1).to(torch.bfloat16)
            w1 = torch.randn(C // 4, C, device=dev) * 0.1
            w2 = torch.randn(C, C // 4, device=dev) * 0.1
            t2 = timeit(lambda: K.linear(K.se_fwd(a2, Fn, HW, C, w1, w2, act=act)[0], w), args.iters)
            t3 = timeit(lambda: K.linear_se(a2, w, act, K.se_fwd(a2, Fn, HW, C, w1, w2, act=act, want_y=False)[3],
                                            HW), args.iters)
            t4 = timeit(lambda: K.se_fwd(a2, Fn, HW, C, w1, w2, act=act, want_y=False), args.iters)
            gate = K.se_fwd(a2, Fn, HW, C, w1, w2, act=act, want_y=False)[3]
            t5 = timeit(lambda: K.linear_se(a2, w, act, gate, HW), args.iters)
            print(f"{name} fwd: se_fwd + proj {t2:7.3f} ms | se gate + proj(se operand) {t3:7.3f} ms "
                  f"(se gate alone {t4:7.3f} ms; proj(se operand) {t5:7.3f} ms)", flush=True)
        del a2, dy
        torch.cuda.empty_cache()


def gemmk(args):
    """Fixed-cost probe: one output shape, growing K (fwd layout, bf16 out, bias)."""
    M, N = args.batch * 6272, 1152
    for Kd in (64, 128, 256, 384, 768, 1536):
        x = torch.randn(M, Kd, device="cuda").to(torch.bfloat16)
        w = torch.randn(N, Kd, device="cuda").to(torch.bfloat16)
        b = torch.randn(N, device="cuda")
        f = 2.0 * M * N * Kd
        t = timeit(lambda: K.linear(x, w, b), args.iters)
        t0 = timeit(lambda: K.linear(x, w), args.iters)
        gb = (M * Kd + M * N) * 2 / 1e9
        print(f"M={M} N={N} K={Kd}: {t:7.3f} ms {f / t / 1e9:7.1f} TF/s {gb / t:7.1f} TB/s | no-bias {t0:7.3f} ms",
              flush=True)
        del x, w
        torch.cuda.empty_cache()


def gemmw(args):
    """Write-rate probe: the stage-0 expand shape (M = batch*8*112^2 rows, N = 384 bf16 out)
    at tiny K against a plain fill of the same output."""
    M, N = args.batch * 8 * 12544, 384
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    gbw = M * N * 2 / 1e9
    t = timeit(lambda: out.zero_(), args.iters)
    print(f"fill [M={M}, {N}] bf16: {t:7.3f} ms  {gbw / t:6.2f} TB/s written", flush=True)
    del out
    # the same bytes written as N = 128 (one n-tile per row: each block writes whole rows)
    x = torch.randn(3 * M, 8, device="cuda").to(torch.bfloat16)
    w = torch.randn(128, 8, device="cuda").to(torch.bfloat16)
    t = timeit(lambda: K.linear(x, w), args.iters)
    print(f"linear M={3 * M} N=128 K=8: {t:7.3f} ms  {gbw / t:6.2f} TB/s written", flush=True)
    del x, w
    torch.cuda.empty_cache()
    for Kd in (8, 32, 96):
        x = torch.randn(M, Kd, device="cuda").to(torch.bfloat16)
        w = torch.randn(N, Kd, device="cuda").to(torch.bfloat16)
        t = timeit(lambda: K.linear(x, w), args.iters)
        gbr = M * Kd * 2 / 1e9
        print(f"linear M={M} N={N} K={Kd}: {t:7.3f} ms  {gbw / t:6.2f} TB/s written, {gbr / t:6.2f} read",
              flush=True)
        del x, w
        torch.cuda.empty_cache()


def stem(args):
    """PatchEmbed forward pieces at B clips of 8x224^2 (bf16), HIP-event timed."""
    dev = "cuda"
    clip = torch.randn(args.batch, 3, 8, 224, 224, device=dev)
    w1p = K.conv_wpack(torch.randn(48, 3, 3, 3, device=dev) * 0.2, 32, 0, torch.bfloat16)
    w2p = K.conv_wpack(torch.randn(96, 48, 3, 3, device=dev) * 0.05, 432, 1, torch.bfloat16)
    g1, b1 = torch.rand(48, device=dev) + 0.5, torch.randn(48, device=dev) * 0.1
    g2, b2 = torch.rand(96, device=dev) + 0.5, torch.randn(96, device=dev) * 0.1
    Fr, Ho, Wo = args.batch * 8, 112, 112

    def rep(name, ms):
        print(f"{name:34s} {ms:8.3f} ms", flush=True)
    rep("stem_im2col", timeit(lambda: K.stem_im2col(clip, torch.bfloat16), args.iters))
    col, _ = K.stem_im2col(clip, torch.bfloat16)
    rep("conv1 GEMM + BN1 stats (im2col in)", timeit(lambda: K.linear_bn_stats(col, w1p), args.iters))
    del col
    rep("stem_conv1_bn_stats (direct)", timeit(lambda: K.stem_conv1_bn_stats(clip, w1p), args.iters))
    a1, m1, r1, _ = K.stem_conv1_bn_stats(clip, w1p)
    rep("stem_conv2_bn_stats (direct, act in ring)",
        timeit(lambda: K.stem_conv2_bn_stats(a1, (m1, r1, g1, b1, True), w2p, Fr, Ho, Wo), args.iters))
    rep("bn_apply + GELU (h1)", timeit(lambda: K.bn_apply(a1, m1, r1, g1, b1, gelu=True), args.iters))
    h1 = K.bn_apply(a1, m1, r1, g1, b1, gelu=True)
    rep("conv3x3_fwd_bn_stats", timeit(lambda: K.conv3x3_fwd_bn_stats(h1, w2p, Fr, Ho, Wo, 48, 96), args.iters))
    a2, m2, r2 = K.conv3x3_fwd_bn_stats(h1, w2p, Fr, Ho, Wo, 48, 96)
    rep("bn_apply (y)", timeit(lambda: K.bn_apply(a2, m2, r2, g2, b2, gelu=False), args.iters))


def mbconv(args):
    """Stage-0 MBConv streaming ops at F = batch*8 frames of 112x112x384 (bf16)."""
    Fn, H, W, C = args.batch * 8, 112, 112, 384
    M = Fn * H * W
    dev = "cuda"
    a = (torch.randn(M, C, device=dev) * 2).to(torch.bfloat16)
    g = torch.rand(C, device=dev) + 0.5
    b = torch.randn(C, device=dev) * 0.1
    m, r = K.bn_stats(a)
    act = (m, r, g, b, True)
    w = torch.randn(C, 9, device=dev) * 0.3

    class BN:
        running_mean = torch.zeros(C, device=dev)
        running_var = torch.ones(C, device=dev)
        num_batches_tracked = torch.zeros((), dtype=torch.int64, device=dev)
        momentum, eps = 0.1, 1e-5
    T = M * C * 2 / 1e9   # GB of one [M][C] bf16 tensor

    def rep(name, ms, passes):
        print(f"{name:28s} {ms:8.2f} ms  {passes * T / ms:6.2f} TB/s ({passes} passes of {T:.1f} GB)", flush=True)
    rep("bn_stats", timeit(lambda: K.bn_stats(a), args.iters), 1)
    rep("bn_apply+gelu", timeit(lambda: K.bn_apply(a, m, r, g, b, gelu=True), args.iters), 2)
    y = K.dwconv_fused(a, act, w, Fn, H, W, C, 1)
    rep("dwconv_fused s1 (+stats)", timeit(lambda: K.dwconv_fused(a, act, w, Fn, H, W, C, 1, bn_out=BN), args.iters), 2)
    rep("dwconv_fused s1 no-act", timeit(lambda: K.dwconv_fused(a, None, w, Fn, H, W, C, 1), args.iters), 2)
    dw = torch.zeros(C, 9, device=dev)
    rep("dwconv_fused_bwd s1", timeit(lambda: K.dwconv_fused_bwd(y, a, act, w, dw, Fn, H, W, C, 1), args.iters), 4)
    g0, b0 = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
    rep("dwconv_bn_bwd s1 (2 passes)", timeit(lambda: K.dwconv_bn_bwd(y, a, act, w, dw, g0, b0, Fn, H, W, C),
                                              args.iters), 5)
    rep("dwconv_fused s2", timeit(lambda: K.dwconv_fused(a, act, w, Fn, H, W, C, 2), args.iters), 1.25)
    y2 = K.dwconv_fused(a, act, w, Fn, H, W, C, 2)
    rep("s2 bwd unfused (dw bwd+bn_bwd)", timeit(lambda: K.bn_bwd(K.dwconv_fused_bwd(y2, a, act, w, dw, Fn, H, W, C, 2),
                                                                  a, m, r, g, b, True, torch.zeros(C, device=dev),
                                                                  torch.zeros(C, device=dev)), args.iters), 5.25)
    rep("dwconv_bn_bwd s2 (2 passes)", timeit(lambda: K.dwconv_bn_bwd(y2, a, act, w, dw, torch.zeros(C, device=dev),
                                                                       torch.zeros(C, device=dev), Fn, H, W, C,
                                                                       stride=2), args.iters), 4.25)
    del y2
    w1 = torch.randn(C // 4, C, device=dev) * 0.1
    w2 = torch.randn(C, C // 4, device=dev) * 0.1
    _, _, h1, sg = K.se_fwd(a, Fn, H * W, C, w1, w2, act=act, want_y=False)
    rep("se_fwd (act)", timeit(lambda: K.se_fwd(a, Fn, H * W, C, w1, w2, act=act), args.iters), 3)
    rep("se_bwd (act)", timeit(lambda: K.se_bwd(y, a, Fn, H * W, C, w1, w2, sg, h1, act=act), args.iters), 4)
    rep("bn_bwd gelu", timeit(lambda: K.bn_bwd(y, a, m, r, g, b, True, torch.zeros(C, device=dev),
                                                torch.zeros(C, device=dev)), args.iters), 5)
    z = torch.zeros(C, device=dev)
    rep("se_bn_bwd (fused)", timeit(lambda: K.se_bn_bwd(y, a, Fn, H * W, C, w1, w2, sg, h1, act, z, z),
                                    args.iters), 5)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("what", choices=["attn", "gemm", "gemmk", "mbconv", "dw", "dwx", "dwse", "stem", "gemmw",
                                     "bnstats", "dxgelu"])
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--drop", type=float, default=0.1)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--only", default="")
    ap.add_argument("--bwd-shapes", default="", help="attn: MFMA shapes of the backward to A/B, e.g. 32,16")
    ap.add_argument("--rounds", type=int, default=1, help="attn / gemm: interleaved rounds per variant")
    ap.add_argument("--mf", default="", help="gemm: K-loop MFMA shapes to A/B, e.g. 32,16")
    a = ap.parse_args()
    from ssl_mae_amd.build import build
    build()
    {"attn": attn, "gemm": gemm, "gemmk": gemmk, "mbconv": mbconv, "dw": dw, "dwx": dwx, "dwse": dwse, "stem": stem, "gemmw": gemmw,
     "bnstats": bnstats, "dxgelu": dxgelu}[a.what](a)
