"""Kernel-level parity on the GPU: every C-ABI entry point against a plain fp32
CPU reference of the same op (torch CPU ops / the oracle).  Tolerances: f32 mode
1e-4-ish relative (exact-fp32 MFMA, different summation order); bf16 mode
compared with the fp32 reference of the SAME bf16-rounded inputs, 2e-2 of scale.
"""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _lib():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from ssl_mae_amd import _lib as L
    L.load()


def KK():
    from ssl_mae_amd import kernels
    return kernels


def rel_err(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return ((a - b).abs().max() / (b.abs().max() + 1e-12)).item()


TOL = {torch.float32: 2e-5, torch.bfloat16: 2e-2}


def drop_scale(p, attn=False):
    """Kept-value scale of the counter-hash dropout (csrc/common.h drop_scale, attention.hip
    attn_drop_scale): the inverse of the quantised keep rate, 256 / (256 - round(256 p)) or
    128 / (128 - round(128 p)), so E[mask * scale] = 1 as nn.Dropout."""
    q = 128 if attn else 256
    return q / (q - int(p * q + 0.5))


def rnd(*shape, dtype=torch.float32, scale=1.0, seed=0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(dtype)


# ------------------------------------------------------------------ GEMM
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("la,lb", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("M,N,K", [(200, 72, 96), (1000, 384, 192), (64, 1152, 384), (256, 96, 8),
                                   # long K with ragged M / N tiles and K tails (not a multiple of 64)
                                   (296, 200, 1088), (520, 96, 1040), (64, 1152, 1024), (768, 512, 1536)])
def test_gemm_layouts(dtype, la, lb, M, N, K):
    A = rnd(M, K, dtype=dtype, seed=1)
    Bm = rnd(K, N, dtype=dtype, seed=2)
    ref = A.float() @ Bm.float()
    a_st = A if la == 0 else A.t().contiguous()        # [M][K] or [K][M]
    b_st = Bm.t().contiguous() if lb == 0 else Bm       # [N][K] or [K][N]
    C = torch.empty(M, N, dtype=dtype, device=DEV)
    KK().gemm(a_st.to(DEV), b_st.to(DEV), C, M, N, K, la, lb, a_st.shape[1], b_st.shape[1], N)
    assert rel_err(C, ref) < TOL[dtype] * (4 if dtype == torch.float32 else 1)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("Kd", [128, 1536])
def test_gemm_epilogues(dtype, Kd):
    M, N = 300, 192
    x = rnd(M, Kd, dtype=dtype, seed=3)
    w = rnd(N, Kd, dtype=dtype, seed=4, scale=0.1)
    b = rnd(N, seed=5)
    r = rnd(M, N, dtype=dtype, seed=6)
    kk = KK()
    y = kk.linear(x.to(DEV), w.to(DEV), b.to(DEV), residual=r.to(DEV))
    ref = x.float() @ w.float().t() + b + r.float()
    assert rel_err(y, ref) < TOL[dtype]
    y, pre = kk.linear(x.to(DEV), w.to(DEV), b.to(DEV), gelu=True)
    refp = x.float() @ w.float().t() + b
    assert rel_err(pre, refp) < TOL[dtype]
    assert rel_err(y, F.gelu(refp)) < TOL[dtype]


def test_gemm_round_branch_residual_fp32():
    M, N, Kd = 128, 384, 384
    x = rnd(M, Kd, dtype=torch.bfloat16, seed=7)
    w = rnd(N, Kd, dtype=torch.bfloat16, seed=8, scale=0.05)
    b = rnd(N, seed=9)
    r = rnd(M, N, seed=10)
    y = KK().linear(x.to(DEV), w.to(DEV), b.to(DEV), out_dtype=torch.float32, residual=r.to(DEV), round_branch=True)
    ref = (x.float() @ w.float().t() + b).bfloat16().float() + r
    assert rel_err(y, ref) < 1e-2


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_gemm_splitk_dw(dtype):
    M, N, Kd = 70000, 96, 384   # dW of a 1x1 conv: reduction over 70k rows -> split-K
    dy = rnd(M, N, dtype=dtype, seed=11, scale=0.1)
    x = rnd(M, Kd, dtype=dtype, seed=12)
    sink = torch.zeros(N, Kd, device=DEV)
    KK().linear_dw(dy.to(DEV), x.to(DEV), sink)
    ref = dy.float().t() @ x.float()
    assert rel_err(sink, ref) < (1e-4 if dtype == torch.float32 else 2e-2)


@pytest.mark.parametrize("M,N,Kd", [(70000, 96, 384), (70000, 384, 1536), (1000, 200, 64), (344, 1152, 384)])
def test_linear_dw_bias_fused(M, N, Kd):
    """dW (+)= dy^T x with db += colsum(dy) from the same GEMM (bf16), split-K and
    single-pass shapes, ragged M-tiles (N = 200: 256-row tile, 56 rows out of range)."""
    dy = rnd(M, N, dtype=torch.bfloat16, seed=14, scale=0.1)
    x = rnd(M, Kd, dtype=torch.bfloat16, seed=15)
    gw = torch.full((N, Kd), 0.25, device=DEV)
    gb = torch.full((N,), -0.5, device=DEV)
    KK().linear_dw_bias(dy.to(DEV), x.to(DEV), gw, gb)
    assert rel_err(gw - 0.25, dy.float().t() @ x.float()) < 2e-2
    assert rel_err(gb + 0.5, dy.float().sum(0)) < 1e-4


def test_colsum():
    x = rnd(5000, 384, seed=13)
    out = torch.ones(384, device=DEV)
    KK().colsum(x.to(DEV), out, accumulate=True)
    assert rel_err(out, x.sum(0) + 1) < 1e-5


# ------------------------------------------------------------------ attention
def _attn_ref(qkv, N, L, H, D):
    qkv = qkv.float().reshape(N, L, 3, H, D).permute(2, 0, 3, 1, 4)
    q, k, v = [t.detach().clone().requires_grad_(True) for t in qkv]
    o = F.scaled_dot_product_attention(q, k, v)
    return q, k, v, o


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("D", [32, 64])
@pytest.mark.parametrize("L", [50, 128, 150, 200])
def test_attention_fwd_bwd(dtype, D, L):
    N, H = 2, 3
    qkv = rnd(N * L, 3 * H * D, dtype=dtype, seed=20 + L + D)
    dO = rnd(N * L, H * D, dtype=dtype, seed=21 + L + D)
    q, k, v, o_ref = _attn_ref(qkv, N, L, H, D)
    o_ref_flat = o_ref.transpose(1, 2).reshape(N * L, H * D)
    o_ref_flat.backward(dO.float())
    dqkv_ref = torch.stack([q.grad, k.grad, v.grad]).permute(1, 3, 0, 2, 4).reshape(N * L, 3 * H * D)
    kk = KK()
    o, lse = kk.attn_fwd(qkv.to(DEV), N, L, H, D)
    assert rel_err(o, o_ref_flat) < TOL[dtype]
    s = (q.detach() @ k.detach().transpose(-1, -2)) / math.sqrt(D)
    lse_ref = torch.logsumexp(s, -1)
    assert rel_err(lse, lse_ref) < (1e-5 if dtype == torch.float32 else 2e-2)
    dqkv = kk.attn_bwd(qkv.to(DEV), o, dO.to(DEV), lse, N, L, H, D)
    assert rel_err(dqkv, dqkv_ref) < (1e-4 if dtype == torch.float32 else 3e-2)


@pytest.mark.parametrize("D", [32, 64])
@pytest.mark.parametrize("case", ["overflow", "underflow"])
def test_attention_fwd_outside_fast_range(D, case):
    """The bf16 forward's max-free pass (P = exp2(S), Q pre-scaled by scale*log2 e) is
    only valid while every row sum stays in [2^-100, 2^100]; rows beyond it must make
    their block rerun with the online softmax.  overflow: sample 0's q, k scaled so the
    log2 scores reach ~150 (sample 1 stays on the fast pass); underflow: every score of
    a row below -130 (q = a u, k = -a u).  Reference: fp32 softmax over the same
    bf16(q * scale * log2 e) scores."""
    N, L, H = 2, 200, 3
    g = torch.Generator().manual_seed(70 + D)
    x = torch.randn(N * L, 3 * H * D, generator=g)
    if case == "overflow":
        x[:L, :2 * H * D] *= 6.0
    else:
        u = torch.randn(H * D, generator=g)
        x[:, :H * D] = 5.0 * u + 0.5 * x[:, :H * D]
        x[:, H * D:2 * H * D] = -5.0 * u + 0.5 * x[:, H * D:2 * H * D]
    qkv = x.to(torch.bfloat16)
    q, k, v = qkv.float().reshape(N, L, 3, H, D).permute(2, 0, 3, 1, 4)
    c = math.log2(math.e) / math.sqrt(D)
    s2 = (q * c).to(torch.bfloat16).float() @ k.transpose(-1, -2)   # log2 units
    o_ref = torch.softmax(s2 * math.log(2.0), -1) @ v
    o_ref_flat = o_ref.transpose(1, 2).reshape(N * L, H * D)
    lse_ref = torch.logsumexp(s2 * math.log(2.0), -1)
    if case == "overflow":
        assert s2[0].max() > 128   # the fast pass overflows here
    else:
        assert s2.max() < -100     # and underflows here
    o, lse = KK().attn_fwd(qkv.to(DEV), N, L, H, D)
    assert torch.isfinite(o.float()).all()
    assert rel_err(o, o_ref_flat) < TOL[torch.bfloat16]
    assert rel_err(lse, lse_ref) < 1e-3


def test_attention_dropout_statistics():
    """Dropout on P: E[O] unchanged; the same seed gives the same output."""
    N, L, H, D = 1, 256, 2, 64
    qkv = rnd(N * L, 3 * H * D, dtype=torch.bfloat16, seed=30).to(DEV)
    kk = KK()
    o0, _ = kk.attn_fwd(qkv, N, L, H, D)
    outs = [kk.attn_fwd(qkv, N, L, H, D, drop_p=0.1, seed=s)[0].float() for s in range(256)]
    again = kk.attn_fwd(qkv, N, L, H, D, drop_p=0.1, seed=0)[0].float()
    assert torch.equal(outs[0], again)
    mean = torch.stack(outs).mean(0)
    assert rel_err(mean, o0.float()) < 0.1   # ~0.05 expected at 256 samples


def _np_keep(rows, cols, p, seed, attn=False):
    """numpy restatement of csrc/common.h drop_keep (counter hash, 8-bit threshold,
    one hash per 4 columns): keep[row, col] for the given index vectors.  attn=True:
    the attention kernels' rule (csrc/attention.hip): mix24 instead of fmix32 and a
    7-bit threshold, (byte & 0x7F) >= round(128 p)."""
    M = 0xFFFFFFFF
    s32 = (seed & M) ^ (seed >> 32)
    r = rows.astype(np.uint64)[:, None]
    c = cols.astype(np.uint64)[None, :]
    h = (s32 + r * 0x9E3779B1 + (c >> 2) * 0x7FEB352D) & M
    if attn:
        h ^= h >> 16; h = ((h & 0xFFFFFF) * 0xEBCA6B) & M
        h ^= h >> 13; h = ((h & 0xFFFFFF) * 0xB2AE35) & M
    else:
        h ^= h >> 16; h = (h * 0x85EBCA6B) & M
        h ^= h >> 13; h = (h * 0xC2B2AE35) & M
    h ^= h >> 16
    byte = (h >> ((c & 3) * 8)) & 0xFF
    if attn:
        return (byte & 0x7F) >= int(p * 128 + 0.5)
    return byte >= int(p * 256 + 0.5)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("D,L", [(64, 200), (32, 130)])
def test_attention_dropout_exact_mask(dtype, D, L):
    """Attention with dropout equals an fp32 torch reference that applies the
    counter-hash mask regenerated on the host -- forward and all three gradients
    (checks the fwd, dK/dV and dQ kernels regenerate the identical mask)."""
    N, H, p, seed = 2, 3, 0.1, 987654321
    qkv = rnd(N * L, 3 * H * D, dtype=dtype, seed=60 + L)
    dO = rnd(N * L, H * D, dtype=dtype, seed=61 + L)
    q, k, v = [t.detach().clone().requires_grad_(True)
               for t in qkv.float().reshape(N, L, 3, H, D).permute(2, 0, 3, 1, 4)]
    rows = np.arange(N * H * L)
    keep = torch.from_numpy(_np_keep(rows, np.arange(L), p, seed, attn=True)).reshape(N, H, L, L)
    P = torch.softmax((q @ k.transpose(-1, -2)) / math.sqrt(D), -1)
    o_ref = (P * keep * drop_scale(p, attn=True)) @ v
    o_ref_flat = o_ref.transpose(1, 2).reshape(N * L, H * D)
    o_ref_flat.backward(dO.float())
    dqkv_ref = torch.stack([q.grad, k.grad, v.grad]).permute(1, 3, 0, 2, 4).reshape(N * L, 3 * H * D)
    kk = KK()
    o, lse = kk.attn_fwd(qkv.to(DEV), N, L, H, D, drop_p=p, seed=seed)
    assert rel_err(o, o_ref_flat) < TOL[dtype]
    dqkv = kk.attn_bwd(qkv.to(DEV), o, dO.to(DEV), lse, N, L, H, D, p, seed)
    assert rel_err(dqkv, dqkv_ref) < (1e-4 if dtype == torch.float32 else 3e-2)


# ------------------------------------------------------------------ LayerNorm
@pytest.mark.parametrize("xd,yd", [(torch.float32, torch.float32), (torch.bfloat16, torch.bfloat16),
                                   (torch.float32, torch.bfloat16)])
@pytest.mark.parametrize("C", [192, 384])
def test_layernorm(xd, yd, C):
    M = 777
    x = (rnd(M, C, seed=40) * 3 + 1).to(xd)
    g = rnd(C, seed=41) * 0.1 + 1
    b = rnd(C, seed=42) * 0.1
    dy = rnd(M, C, seed=43).to(yd)
    xr = x.float().requires_grad_(True)
    gr = g.clone().requires_grad_(True)
    br = b.clone().requires_grad_(True)
    yr = F.layer_norm(xr, (C,), gr, br, 1e-5)
    yr.backward(dy.float())
    kk = KK()
    y, mean, rstd = kk.layernorm(x.to(DEV), g.to(DEV), b.to(DEV), out_dtype=yd)
    tol = 2e-5 if yd == torch.float32 else 1e-2
    assert rel_err(y, yr) < tol
    dg = torch.zeros(C, device=DEV)
    db = torch.zeros(C, device=DEV)
    res = rnd(M, C, seed=44).to(xd)
    dx = kk.layernorm_bwd(dy.to(DEV), x.to(DEV), mean, rstd, g.to(DEV), dg, db, dres=res.to(DEV))
    tol = 1e-4 if xd == torch.float32 and yd == torch.float32 else 2e-2
    assert rel_err(dx, xr.grad + res.float()) < tol
    assert rel_err(dg, gr.grad) < 1e-4
    assert rel_err(db, br.grad) < 1e-4


@pytest.mark.parametrize("xd,p,rs,C", [(torch.float32, 0.1, False, 384), (torch.float32, 0.0, False, 384),
                                       (torch.bfloat16, 0.0, True, 384), (torch.bfloat16, 0.0, True, 192),
                                       (torch.float32, 0.1, True, 192), (torch.bfloat16, 0.1, False, 384)])
def test_layernorm_bwd_branch(xd, p, rs, C):
    """LayerNorm backward with the block branch's bf16 copy of dx (sm_layernorm_bwd_branch):
    dx and the weight gradients bit-identical to sm_layernorm_bwd, the copy bit-identical
    to cast + dropout_bwd (dropout mask, DropPath row scale per group of rows); and the
    fused fp32 -> bf16 cast + dropout backward (sm_cast_dropout_bwd) bit-identical to the
    two passes."""
    kk = KK()
    M, L = 777, 37
    x = ((rnd(M, C, seed=45) * 3 + 1).to(xd)).to(DEV)
    g = (rnd(C, seed=46) * 0.1 + 1).to(DEV)
    b = (rnd(C, seed=47) * 0.1).to(DEV)
    dy = rnd(M, C, seed=48).to(torch.bfloat16).to(DEV)
    res = rnd(M, C, seed=49).to(xd).to(DEV)
    _, mean, rstd = kk.layernorm(x, g, b, out_dtype=torch.bfloat16)
    row_scale = kk.droppath_scale((M + L - 1) // L, 0.2, 1234, DEV) if rs else None
    dg1, db1 = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
    dg2, db2 = dg1.clone(), db1.clone()
    dx1 = kk.layernorm_bwd(dy, x, mean, rstd, g, dg1, db1, dres=res)
    ref = dx1 if xd == torch.bfloat16 else kk.cast(dx1, torch.bfloat16)
    ref = kk.dropout_bwd(ref, p, 99, row_scale, L)
    dx2, dxb = kk.layernorm_bwd_branch(dy, x, mean, rstd, g, dg2, db2, dres=res, drop_p=p, seed=99,
                                       row_scale=row_scale, rows_per_group=L)
    assert torch.equal(dx1, dx2) and torch.equal(dg1, dg2) and torch.equal(db1, db2)
    assert dxb.dtype == torch.bfloat16 and torch.equal(dxb, ref)
    if xd == torch.float32:
        fused = kk.cast_dropout_bwd(dx1, p, 99, row_scale, L)
        assert torch.equal(fused, ref)


# ------------------------------------------------------------------ BatchNorm
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("C", [48, 96, 384, 768])
@pytest.mark.parametrize("gelu", [False, True])
def test_batchnorm_train(dtype, C, gelu):
    M = 3000
    x = (rnd(M, C, seed=50) * 2 + 0.5).to(dtype)
    w = rnd(C, seed=51) * 0.1 + 1
    b = rnd(C, seed=52) * 0.1
    dy = rnd(M, C, seed=53).to(dtype)
    xr = x.float().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    br = b.clone().requires_grad_(True)
    rm_ref = torch.zeros(C)
    rv_ref = torch.ones(C)
    yr = F.batch_norm(xr, rm_ref, rv_ref, wr, br, True, 0.1, 1e-5)
    if gelu:
        yr = F.gelu(yr)
    yr.backward(dy.float())
    kk = KK()
    rm = torch.zeros(C, device=DEV)
    rv = torch.ones(C, device=DEV)
    xd = x.to(DEV)
    mean, rstd = kk.bn_stats(xd, rm, rv)
    assert rel_err(rm, rm_ref) < 1e-4 and rel_err(rv, rv_ref) < 1e-4
    y = kk.bn_apply(xd, mean, rstd, w.to(DEV), b.to(DEV), gelu=gelu)
    assert rel_err(y, yr) < TOL[dtype] * 2
    dw = torch.zeros(C, device=DEV)
    db = torch.zeros(C, device=DEV)
    dx = kk.bn_bwd(dy.to(DEV), xd, mean, rstd, w.to(DEV), b.to(DEV), gelu, dw, db)
    assert rel_err(dx, xr.grad) < (1e-4 if dtype == torch.float32 else 3e-2)
    assert rel_err(dw, wr.grad) < (1e-4 if dtype == torch.float32 else 2e-2)
    assert rel_err(db, br.grad) < 1e-4


# ------------------------------------------------------------------ convs
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("stride", [1, 2])
def test_dwconv(dtype, stride):
    Fn, H, W, C = 3, 14, 12, 64
    x = rnd(Fn, H, W, C, dtype=dtype, seed=60)
    w = rnd(C, 1, 3, 3, seed=61) * 0.3
    xr = x.float().permute(0, 3, 1, 2).contiguous().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    yr = F.conv2d(xr, wr, None, stride, 1, 1, C)
    dy = rnd(*yr.shape, seed=62).to(dtype).float()
    yr.backward(dy)
    kk = KK()
    y = kk.dwconv(x.to(DEV).reshape(-1, C), w.to(DEV).reshape(C, 9), Fn, H, W, C, stride)
    assert rel_err(y, yr.permute(0, 2, 3, 1).reshape(-1, C)) < TOL[dtype]
    dw = torch.zeros(C, 9, device=DEV)
    dyd = dy.permute(0, 2, 3, 1).reshape(-1, C).to(dtype).to(DEV)
    dx = kk.dwconv_bwd(dyd, x.to(DEV).reshape(-1, C), w.to(DEV).reshape(C, 9), dw, Fn, H, W, C, stride)
    assert rel_err(dx, xr.grad.permute(0, 2, 3, 1).reshape(-1, C)) < TOL[dtype]
    assert rel_err(dw, wr.grad.reshape(C, 9)) < (1e-4 if dtype == torch.float32 else 2e-2)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_stem_conv_via_im2col(dtype):
    B, T, S = 2, 3, 32
    clip = rnd(B, 3, T, S, S, seed=70)
    w1 = rnd(48, 3, 3, 3, seed=71) * 0.2
    kk = KK()
    col, (Fn, Ho, Wo) = kk.stem_im2col(clip.to(DEV), dtype)
    w1p = kk.conv_wpack(w1.to(DEV), 32, 0, dtype)
    y = kk.linear(col, w1p)
    frames = clip.permute(0, 2, 1, 3, 4).reshape(B * T, 3, S, S)
    ref = F.conv2d(frames.to(dtype).float(), w1, None, 2, 1).permute(0, 2, 3, 1).reshape(-1, 48)
    assert rel_err(y, ref) < TOL[dtype] * 2
    # conv2 48->96 k3 s1 via im2col3 + GEMM, and its dgrad via col2im3
    x2 = rnd(Fn, Ho, Wo, 48, dtype=dtype, seed=72)
    w2 = rnd(96, 48, 3, 3, seed=73) * 0.05
    col2 = kk.im2col3(x2.to(DEV).reshape(-1, 48), Fn, Ho, Wo, 48, 1)
    w2p = kk.conv_wpack(w2.to(DEV), 432, 1, dtype)
    y2 = kk.linear(col2, w2p)
    xr = x2.float().permute(0, 3, 1, 2).contiguous().requires_grad_(True)
    wr = w2.clone().requires_grad_(True)
    ref2 = F.conv2d(xr, wr, None, 1, 1)
    assert rel_err(y2, ref2.permute(0, 2, 3, 1).reshape(-1, 96)) < TOL[dtype] * 2
    dy = rnd(*ref2.shape, seed=74).to(dtype).float()
    ref2.backward(dy)
    dyd = dy.permute(0, 2, 3, 1).reshape(-1, 96).to(dtype).to(DEV)
    dcol = kk.linear_dx(dyd, w2p)
    dx = kk.col2im3(dcol, Fn, Ho, Wo, 48, 1)
    assert rel_err(dx, xr.grad.permute(0, 2, 3, 1).reshape(-1, 48)) < TOL[dtype] * 2
    dwp = torch.zeros(96, 432, device=DEV)
    kk.linear_dw(dyd, col2, dwp)
    g = torch.zeros(96, 48, 3, 3, device=DEV)
    kk.conv_wunpack_add(dwp, g, 1)
    assert rel_err(g, wr.grad) < (1e-4 if dtype == torch.float32 else 2e-2)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_se_layer(dtype):
    Fn, HW, C = 4, 49, 96
    R = C // 4
    x = rnd(Fn, HW, C, dtype=dtype, seed=80)
    w1 = rnd(R, C, seed=81) * 0.2
    w2 = rnd(C, R, seed=82) * 0.2
    xr = x.float().requires_grad_(True)
    w1r = w1.clone().requires_grad_(True)
    w2r = w2.clone().requires_grad_(True)
    p = xr.mean(1)
    h = torch.relu(p @ w1r.t())
    s = torch.sigmoid(h @ w2r.t())
    yr = xr * s[:, None, :]
    dy = rnd(Fn, HW, C, seed=83).to(dtype).float()
    yr.backward(dy)
    kk = KK()
    y, pooled, h1, sd = kk.se_fwd(x.to(DEV).reshape(-1, C), Fn, HW, C, w1.to(DEV), w2.to(DEV))
    assert rel_err(y, yr.reshape(-1, C)) < TOL[dtype]
    dx, dz2, dz1 = kk.se_bwd(dy.to(dtype).to(DEV).reshape(-1, C), x.to(DEV).reshape(-1, C), Fn, HW, C,
                             w1.to(DEV), w2.to(DEV), sd, h1)
    assert rel_err(dx, xr.grad.reshape(-1, C)) < TOL[dtype] * 2
    dw2 = torch.zeros(C, R, device=DEV)
    KK().gemm(dz2, h1, dw2, C, R, Fn, 1, 1, C, R, R, beta=1.0)
    dw1 = torch.zeros(R, C, device=DEV)
    KK().gemm(dz1, pooled, dw1, R, C, Fn, 1, 1, R, C, C, beta=1.0)
    assert rel_err(dw2, w2r.grad) < (1e-4 if dtype == torch.float32 else 2e-2)
    assert rel_err(dw1, w1r.grad) < (1e-4 if dtype == torch.float32 else 2e-2)


# ------------------------------------------------------------------ fused MBConv depthwise / SE paths
class _BN:
    def __init__(self, C):
        self.running_mean = torch.zeros(C, device=DEV)
        self.running_var = torch.ones(C, device=DEV)
        self.num_batches_tracked = torch.zeros((), dtype=torch.int64, device=DEV)
        self.momentum, self.eps = 0.1, 1e-5


def _act_for(a2d, seed):
    """BN(train) + GELU parameters of a [M][C] pre-activation (the MBConv producer)."""
    kk = KK()
    C = a2d.shape[1]
    g = (rnd(C, seed=seed) * 0.2 + 1).to(DEV)
    b = (rnd(C, seed=seed + 1) * 0.2).to(DEV)
    m, r = kk.bn_stats(a2d)
    return (m, r, g, b, True)


@pytest.mark.parametrize("stride,H,W,C", [(1, 14, 14, 64), (1, 9, 23, 32), (2, 14, 14, 64), (2, 13, 11, 96)])
def test_dwconv_fused_matches_unfused(stride, H, W, C):
    """dwconv(act(x)) with act folded into the loads == bn_apply + dwconv (bit-exact y);
    in-kernel BN statistics == a separate bn_stats pass; backward (dx, dw) == the
    unfused backward on the materialised act(x)."""
    kk = KK()
    Fn = 3
    a = (rnd(Fn * H * W, C, seed=90) * 2 + 0.5).to(torch.bfloat16).to(DEV)
    w = (rnd(C, 9, seed=91) * 0.3).to(DEV)
    act = _act_for(a, 92)
    h = kk.bn_apply(a, act[0], act[1], act[2], act[3], gelu=True)
    y_ref = kk.dwconv(h, w, Fn, H, W, C, stride)
    bn_f, bn_r = _BN(C), _BN(C)
    y, mean, rstd = kk.dwconv_fused(a, act, w, Fn, H, W, C, stride, bn_out=bn_f)
    assert torch.equal(y, y_ref)
    m_ref, r_ref = kk.bn_stats(y_ref, bn_r.running_mean, bn_r.running_var, 0.1, 1e-5, 1, bn_r.num_batches_tracked)
    assert rel_err(mean, m_ref) < 1e-5 and rel_err(rstd, r_ref) < 1e-5
    assert rel_err(bn_f.running_var, bn_r.running_var) < 1e-5 and int(bn_f.num_batches_tracked) == 1
    dy = rnd(*y.shape, seed=93).to(torch.bfloat16).to(DEV)
    dw_ref = torch.zeros(C, 9, device=DEV)
    dx_ref = kk.dwconv_bwd(dy, h, w, dw_ref, Fn, H, W, C, stride)
    dw = torch.zeros(C, 9, device=DEV)
    dx = kk.dwconv_fused_bwd(dy, a, act, w, dw, Fn, H, W, C, stride)
    assert rel_err(dx, dx_ref) < 1e-2
    assert rel_err(dw, dw_ref) < 1e-4


@pytest.mark.parametrize("HW,C", [(49, 96), (900, 64), (1600, 384)])
def test_se_fused_act_matches_materialised(HW, C):
    """SE on act(x) recomputed in its kernels == SE on the materialised act(x)."""
    kk = KK()
    Fn, R = 3, C // 4
    a = (rnd(Fn * HW, C, seed=95) * 2).to(torch.bfloat16).to(DEV)
    act = _act_for(a, 96)
    h = kk.bn_apply(a, act[0], act[1], act[2], act[3], gelu=True)
    w1 = (rnd(R, C, seed=97) * 0.2).to(DEV)
    w2 = (rnd(C, R, seed=98) * 0.2).to(DEV)
    y_r, p_r, h1_r, s_r = kk.se_fwd(h, Fn, HW, C, w1, w2)
    y, p, h1, s = kk.se_fwd(a, Fn, HW, C, w1, w2, act=act)
    assert rel_err(p, p_r) < 1e-5 and rel_err(s, s_r) < 1e-5
    assert rel_err(y, y_r) < 1e-2
    assert torch.equal(kk.se_scale(a, s, Fn, HW, C, act=act), kk.se_scale(h, s, Fn, HW, C))
    dy = rnd(Fn * HW, C, seed=99).to(torch.bfloat16).to(DEV)
    dx_r, dz2_r, dz1_r = kk.se_bwd(dy, h, Fn, HW, C, w1, w2, s, h1)
    dx, dz2, dz1 = kk.se_bwd(dy, a, Fn, HW, C, w1, w2, s, h1, act=act)
    assert rel_err(dz2, dz2_r) < 1e-5 and rel_err(dz1, dz1_r) < 1e-5
    assert rel_err(dx, dx_r) < 1e-2


@pytest.mark.parametrize("HW,C", [(49, 96), (1000, 384)])
def test_se_bn_bwd_fused_matches_composition(HW, C):
    """Fused SE + BN2/GELU backward == se_bwd followed by bn_bwd(gelu) on its dx
    (the composed path rounds dh2 to bf16 in HBM; the fused one keeps it in fp32)."""
    kk = KK()
    Fn, R = 3, C // 4
    a = (rnd(Fn * HW, C, seed=105) * 2).to(torch.bfloat16).to(DEV)
    act = _act_for(a, 106)
    w1 = (rnd(R, C, seed=107) * 0.2).to(DEV)
    w2 = (rnd(C, R, seed=108) * 0.2).to(DEV)
    _, _, h1, s = kk.se_fwd(a, Fn, HW, C, w1, w2, act=act)
    dy = rnd(Fn * HW, C, seed=109).to(torch.bfloat16).to(DEV)
    dh2, dz2_r, dz1_r = kk.se_bwd(dy, a, Fn, HW, C, w1, w2, s, h1, act=act)
    dw_r, db_r = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
    dx_r = kk.bn_bwd(dh2, a, act[0], act[1], act[2], act[3], True, dw_r, db_r)
    dw, db = torch.full((C,), 0.5, device=DEV), torch.full((C,), -0.5, device=DEV)
    dx, dz2, dz1 = kk.se_bn_bwd(dy, a, Fn, HW, C, w1, w2, s, h1, act, dw, db)
    assert rel_err(dz2, dz2_r) < 1e-5 and rel_err(dz1, dz1_r) < 1e-5
    assert rel_err(dw - 0.5, dw_r) < 5e-3 and rel_err(db + 0.5, db_r) < 5e-3
    assert rel_err(dx, dx_r) < 1e-2


# ------------------------------------------------------------------ MAE glue
def test_tube_mask_and_gather_bit_exact():
    from oracle import mae_oracle as O
    B, T, L, r = 16, 8, 784, 0.75
    n_mask = int(r * L)
    torch.manual_seed(7)
    ref = O.get_tube_mask(B, T, L, r)
    torch.manual_seed(7)
    noise = torch.stack([torch.rand(L) for _ in range(B)])
    mask, idx = KK().tube_mask(noise.to(DEV), T, n_mask)
    assert torch.equal(mask.cpu().bool(), ref)
    ref_idx = torch.nonzero(ref.reshape(-1)).reshape(-1).int()
    assert torch.equal(idx.cpu(), ref_idx)
    pred = rnd(B * T * L, 192, dtype=torch.bfloat16, seed=90)
    g = KK().gather_rows(pred.to(DEV), idx)
    assert torch.equal(g.cpu(), pred[ref.reshape(-1)])
    sd = KK().std(g)
    assert abs(sd.item() - pred[ref.reshape(-1)].float().std().item()) < 1e-4


def test_tube_mask_constructed_cut_ties():
    """Equal noise values straddling the int(r*L) cut: the host tie resolution +
    sm_tube_mask select exactly the reference's argsort(descending)[:n] (mae_loader.py:86)
    and emit the row-major index list of that mask."""
    from test_tube_mask_cpu import constructed_cut_ties, reference_select
    from ssl_mae_amd.mae_loader import tube_mask_from_noise
    B, T, L, nm = 32, 8, 784, 588
    noise = constructed_cut_ties(B, L, nm, seed=11)
    noise[5] = torch.rand(L)                 # a row with no tie at the cut
    mask, idx = tube_mask_from_noise(noise, T, nm, DEV)
    ref = torch.stack([torch.from_numpy(reference_select(noise[b], nm)) for b in range(B)])
    ref = ref[:, None, :].expand(B, T, L).contiguous()
    assert torch.equal(mask.cpu(), ref)
    assert torch.equal(idx.cpu(), torch.nonzero(ref.reshape(-1)).reshape(-1).int())


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_mae_loss(dtype):
    from oracle import mae_oracle as O
    B, T, S = 2, 3, 32
    L = (S // 8) ** 2
    clip = rnd(B, 3, T, S, S, seed=100)
    torch.manual_seed(3)
    mask = O.get_tube_mask(B, T, L, 0.75)
    pred = rnd(B, T * L, 192, dtype=dtype, seed=101)
    pr = pred.float().requires_grad_(True)
    tgt = O.norm_pix(O.patchify(clip, 8))
    lr_ = O.masked_mse(pr, tgt, mask)
    lr_.backward()
    kk = KK()
    m8 = mask.to(torch.uint8).to(DEV)
    loss, denom = kk.mae_loss_fwd(pred.to(DEV), clip.to(DEV), m8)
    assert abs(loss.item() - lr_.item()) < 1e-5 * max(1, abs(lr_.item()))
    g = torch.ones((), device=DEV)
    dpred = kk.mae_loss_bwd(pred.to(DEV), clip.to(DEV), m8, True, g, denom)
    assert rel_err(dpred, pr.grad) < (1e-5 if dtype == torch.float32 else 1e-2)


def test_pos_blend():
    B, T, L, D = 2, 3, 16, 384
    y = rnd(B * T * L, D, dtype=torch.bfloat16, seed=110)
    tpos = rnd(1, T, 1, D, seed=111) * 0.02
    spos = rnd(1, 1, L, D, seed=112) * 0.02
    tok = rnd(1, 1, D, seed=113) * 0.02
    torch.manual_seed(0)
    mask = torch.rand(B, T, L) < 0.5
    yr = y.float().requires_grad_(True)
    tr = tpos.clone().requires_grad_(True)
    sr = spos.clone().requires_grad_(True)
    kr = tok.clone().requires_grad_(True)
    x = yr.reshape(B, T, L, D) + (tr + sr)
    m = mask.float()[..., None]
    x = x * (1 - m) + kr * m
    dx = rnd(B, T, L, D, seed=114)
    x.backward(dx)
    kk = KK()
    m8 = mask.to(torch.uint8).to(DEV)
    out = kk.pos_blend(y.to(DEV), tpos.to(DEV).reshape(T, D), spos.to(DEV).reshape(L, D), tok.to(DEV).reshape(D),
                       m8, B, T, L, D, torch.float32)
    assert rel_err(out, x.reshape(-1, D)) < 1e-6
    dt_ = torch.zeros(T, D, device=DEV)
    ds_ = torch.zeros(L, D, device=DEV)
    dk_ = torch.zeros(D, device=DEV)
    dy = kk.pos_blend_bwd(dx.reshape(-1, D).to(DEV), m8, torch.bfloat16, dt_, ds_, dk_, B, T, L, D)
    assert rel_err(dy, yr.grad.reshape(-1, D)) < 1e-2
    assert rel_err(dt_, tr.grad.reshape(T, D)) < 1e-5
    assert rel_err(ds_, sr.grad.reshape(L, D)) < 1e-5
    assert rel_err(dk_, kr.grad.reshape(D)) < 1e-5


def test_adamw_matches_torch():
    n = 10000
    p0 = rnd(n, seed=120)
    grads = [rnd(n, seed=121 + i) * 0.01 for i in range(3)]
    pr = p0.clone().requires_grad_(True)
    opt = torch.optim.AdamW([pr], lr=5e-4, weight_decay=0.05)
    for g in grads:
        pr.grad = g.clone()
        opt.step()
    kk = KK()
    p = p0.to(DEV)
    m = torch.zeros(n, device=DEV)
    v = torch.zeros(n, device=DEV)
    flag = torch.zeros(1, dtype=torch.int32, device=DEV)
    step = torch.zeros(1, dtype=torch.int64, device=DEV)
    for g in grads:
        gd = g.to(DEV)
        flag.zero_()
        kk.nonfinite(gd, flag)
        kk.adamw(p, gd, m, v, 5e-4, 0.9, 0.999, 1e-8, 0.05, flag, step)
    assert rel_err(p, pr.detach()) < 1e-6
    bad = grads[0].clone().to(DEV)
    bad[5] = float("nan")
    flag.zero_()
    kk.nonfinite(bad, flag)
    before = p.clone()
    kk.adamw(p, bad, m, v, 5e-4, 0.9, 0.999, 1e-8, 0.05, flag, step)
    assert torch.equal(p, before) and step.item() == 3


def test_dropout_masks_fwd_bwd_consistent():
    """GEMM-epilogue dropout, GELU dropout and their backward kernels regenerate the
    same counter-hash mask; keep rate ~ 1-p; kept entries scaled by 256/(256-round(256p))."""
    kk = KK()
    M, N, Kd, p, seed = 512, 384, 64, 0.1, 1234
    x = rnd(M, Kd, dtype=torch.bfloat16, seed=1).to(DEV)
    w = rnd(N, Kd, dtype=torch.bfloat16, seed=2).to(DEV)
    R = torch.zeros(M, N, dtype=torch.float32, device=DEV)
    y0 = kk.linear(x, w, out_dtype=torch.float32, residual=R)
    y = kk.linear(x, w, out_dtype=torch.float32, residual=R, drop_p=p, seed=seed)
    ratio = (y / y0).cpu()
    kept = (ratio.abs() > 0.5)
    assert abs(kept.float().mean().item() - (1 - p)) < 0.01
    assert torch.allclose(ratio[kept], torch.full_like(ratio[kept], drop_scale(p)), rtol=1e-3)
    g = kk.dropout_bwd(torch.ones(M, N, dtype=torch.float32, device=DEV), p, seed).cpu()
    assert torch.equal(g > 0, kept)
    pre = rnd(M, N, dtype=torch.bfloat16, seed=3).to(DEV)
    h = kk.gelu(pre, p, seed).float().cpu()
    h0 = kk.gelu(pre).float().cpu()
    d = kk.gelu_bwd(pre, torch.ones(M, N, dtype=torch.bfloat16, device=DEV), p, seed).float().cpu()
    km = (h != 0) | (h0 == 0)
    assert torch.equal((d != 0) | (h0 == 0), km)
    s = kk.droppath_scale(10000, 0.1, 7, DEV).cpu()
    vals = torch.unique(s)
    assert len(vals) == 2 and vals[0] == 0 and abs(vals[1].item() - drop_scale(0.1)) < 1e-6
    assert abs((s > 0).float().mean() - 0.9) < 0.02


@pytest.mark.parametrize("dtype,p", [(torch.bfloat16, 0.1), (torch.bfloat16, 0.0), (torch.float32, 0.1)])
def test_linear_dx_gelu_backward_epilogue(dtype, p):
    """fc2's data gradient with GELU' and the fc1 output's dropout mask applied in the
    GEMM epilogue (BlockFn backward) == linear_dx followed by gelu_bwd, and == the fp32
    torch autograd of dropout(GELU(pre)) @ w^T."""
    kk = KK()
    M, N, Kd, seed = 777, 384, 1536, 4321
    dy = rnd(M, N, dtype=dtype, seed=150).to(DEV)
    w = rnd(N, Kd, dtype=dtype, seed=151, scale=0.05).to(DEV)
    pre = rnd(M, Kd, dtype=dtype, seed=152).to(DEV)
    got = kk.linear_dx(dy, w, gelu_pre=pre, drop_p=p, seed=seed)
    ref2 = kk.gelu_bwd(pre, kk.linear_dx(dy, w), p, seed)
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    assert rel_err(got, ref2) < tol
    keep = (kk.gelu(pre, p, seed).float() != 0) | (kk.gelu(pre).float() == 0)
    pr = pre.float().requires_grad_(True)
    h = F.gelu(pr) * keep * drop_scale(p)
    h.backward(dy.float() @ w.float())
    assert rel_err(got, pr.grad) < tol


@pytest.mark.parametrize("M", [98, 49, 1001, 1100, 4099])
def test_weight_grad_any_row_count(M):
    """dW = dy^T x over a token-row count that is not a multiple of 8 (fine-tune
    per-frame calls: B * 7 * 7 rows): both operands M/N-major, K tail zero-filled."""
    dy = rnd(M, 576, dtype=torch.bfloat16, seed=140, scale=0.1)
    x = rnd(M, 1536, dtype=torch.bfloat16, seed=141)
    gw = torch.zeros(576, 1536, device=DEV)
    gb = torch.zeros(576, device=DEV)
    KK().linear_dw_bias(dy.to(DEV), x.to(DEV), gw, gb)
    assert rel_err(gw, dy.float().t() @ x.float()) < 2e-2
    assert rel_err(gb, dy.float().sum(0)) < 1e-4


@pytest.mark.parametrize("C", [48, 1536])
def test_batchnorm_eval_and_wide_channels(C):
    """Eval-mode BN from running statistics (sm_bn_eval_params + bn_apply) and train-mode
    statistics / backward at C = 1536 (stage-4 MBConv: column slices) vs F.batch_norm."""
    kk = KK()
    M = 2000
    x = (rnd(M, C, seed=150) * 2 + 0.5).to(DEV)
    w = (rnd(C, seed=151) * 0.1 + 1).to(DEV)
    b = (rnd(C, seed=152) * 0.1).to(DEV)

    class BN:
        running_mean = (rnd(C, seed=153) * 0.3).to(DEV)
        running_var = (rnd(C, seed=154).abs() + 0.5).to(DEV)
        eps = 1e-5
    m, r = kk.bn_eval_params(BN)
    y = kk.bn_apply(x, m, r, w, b, gelu=True)
    ref = F.gelu(F.batch_norm(x, BN.running_mean, BN.running_var, w, b, False, 0.1, 1e-5))
    assert rel_err(y, ref) < 1e-5
    xr = x.detach().clone().requires_grad_(True)
    rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    yr = F.gelu(F.batch_norm(xr, rm, rv, w, b, True, 0.1, 1e-5))
    dy = rnd(M, C, seed=155).to(DEV)
    yr.backward(dy)
    rm2, rv2 = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    mean, rstd = kk.bn_stats(x, rm2, rv2)
    assert rel_err(rm2, rm) < 1e-5 and rel_err(rv2, rv) < 1e-5
    assert rel_err(kk.bn_apply(x, mean, rstd, w, b, gelu=True), yr) < 1e-5
    dw, db = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
    dx = kk.bn_bwd(dy, x, mean, rstd, w, b, True, dw, db)
    assert rel_err(dx, xr.grad) < 1e-4


def test_segment_mean_fwd_bwd():
    kk = KK()
    G, R, C = 37, 49, 576
    x = rnd(G * R, C, dtype=torch.bfloat16, seed=160).to(DEV)
    out = kk.segment_mean(x, G, R, C)
    assert rel_err(out, x.float().view(G, R, C).mean(1)) < 1e-5
    dy = rnd(G, C, seed=161).to(DEV)
    dx = kk.segment_mean_bwd(dy, G, R, C, torch.bfloat16)
    assert rel_err(dx, (dy / R)[:, None, :].expand(G, R, C).reshape(G * R, C)) < 1e-2


@pytest.mark.parametrize("Fn,H,W,Cin,Cout", [(3, 14, 12, 48, 96), (2, 9, 23, 16, 24), (1, 112, 112, 48, 96)])
def test_conv3x3_implicit_gemm(Fn, H, W, Cin, Cout):
    """Stem conv2 as GEMMs over the implicit im2col (sm_conv3x3_fwd / _dgrad / _wgrad)
    against F.conv2d fp32 autograd from the same bf16 inputs; frame borders, ragged
    row tiles and a pixel count that is not a tile multiple."""
    kk = KK()
    x = rnd(Fn, H, W, Cin, dtype=torch.bfloat16, seed=170)
    w = rnd(Cout, Cin, 3, 3, seed=171) * 0.1
    xr = x.float().permute(0, 3, 1, 2).contiguous().requires_grad_(True)
    wr = w.bfloat16().float().clone().requires_grad_(True)
    yr = F.conv2d(xr, wr, None, 1, 1)
    dy = rnd(*yr.shape, seed=172).to(torch.bfloat16)
    yr.backward(dy.float())
    wd = w.to(DEV)
    y = kk.conv3x3_fwd(x.to(DEV).reshape(-1, Cin), kk.conv_wpack(wd, 9 * Cin, 1, torch.bfloat16), Fn, H, W, Cin, Cout)
    assert rel_err(y, yr.permute(0, 2, 3, 1).reshape(-1, Cout)) < 2e-2
    dyd = dy.permute(0, 2, 3, 1).reshape(-1, Cout).contiguous().to(DEV)
    dx = kk.conv3x3_dgrad(dyd, kk.conv_wpack(wd, 9 * Cout, 2, torch.bfloat16), Fn, H, W, Cin, Cout)
    assert rel_err(dx, xr.grad.permute(0, 2, 3, 1).reshape(-1, Cin)) < 2e-2
    dwp = torch.full((Cout, 9 * Cin), 0.5, device=DEV)
    kk.conv3x3_wgrad(dyd, x.to(DEV).reshape(-1, Cin), dwp, Fn, H, W, Cin, Cout, accumulate=True)
    g = torch.zeros(Cout, Cin, 3, 3, device=DEV)
    kk.conv_wunpack_add(dwp - 0.5, g, 1)
    assert rel_err(g, wr.grad) < 2e-2


@pytest.mark.parametrize("M,N,H,p", [(70000, 256, 1536, 0.1), (70000, 192, 768, 0.0), (1001, 96, 64, 0.1),
                                     (70000, 384, 1536, 0.1)])
def test_linear_dw_bias_gelu_operand(M, N, H, p):
    """fc2's weight gradient of dropout(GELU(pre)): with the activation formed in the
    GEMM's operand loads (N <= 256, no recompute pass) or through the gelu kernel (N =
    384), bit-identical to gelu() + linear_dw_bias(), and the fp32 torch math of the
    same mask."""
    kk = KK()
    pre = rnd(M, H, dtype=torch.bfloat16, seed=170).to(DEV)
    dy = rnd(M, N, dtype=torch.bfloat16, seed=171, scale=0.1).to(DEV)
    h = kk.gelu(pre, p, 99)
    gw1, gb1 = torch.zeros(N, H, device=DEV), torch.zeros(N, device=DEV)
    gw2, gb2 = gw1.clone(), gb1.clone()
    kk.linear_dw_bias(dy, h, gw1, gb1)
    kk.linear_dw_bias(dy, pre, gw2, gb2, gelu=(p, 99))
    assert torch.equal(gw1, gw2) and torch.equal(gb1, gb2)
    keep = ((h.float() != 0) | (kk.gelu(pre).float() == 0)).float()
    ref = dy.float().t() @ (F.gelu(pre.float()) * keep * drop_scale(p))
    assert rel_err(gw2, ref) < 2e-2


@pytest.mark.parametrize("M,N,H,p", [(70000, 384, 1536, 0.1), (1001, 384, 1536, 0.0), (300, 96, 64, 0.1),
                                     (6000, 192, 776, 0.1)])
def test_linear_dx_gelu_side_output(M, N, H, p):
    """fc2's data gradient through dropout(GELU(pre)) with h = dropout(GELU(pre)) as a side
    output of the same epilogue (sm_linear_dx_gelu): dx bit-identical to linear_dx(gelu_pre)
    and h bit-identical to the gelu kernel, at the decoder shape, without dropout, a
    single-tile M and a ragged column tile (H = 776)."""
    kk = KK()
    pre = rnd(M, H, dtype=torch.bfloat16, seed=190).to(DEV)
    dy = rnd(M, N, dtype=torch.bfloat16, seed=191, scale=0.1).to(DEV)
    w = rnd(N, H, dtype=torch.bfloat16, seed=192, scale=0.05).to(DEV)
    dx1 = kk.linear_dx(dy, w, gelu_pre=pre, drop_p=p, seed=77)
    h1 = kk.gelu(pre, p, 77)
    dx2, h2 = kk.linear_dx_gelu(dy, w, pre, p, 77)
    assert torch.equal(dx1, dx2)
    assert torch.equal(h1, h2)


@pytest.mark.parametrize("Fr,HW,N,C,acc", [(3, 64, 96, 384, True), (5, 192, 96, 200, False), (2, 3136, 192, 768, True),
                                           (64, 12544, 96, 384, True), (1, 128, 8, 8, False)])
def test_linear_dw_se_operand(Fr, HW, N, C, acc):
    """MBConv projection weight gradient over the SE output h3 = bf16(bf16(GELU(BN(a2)))
    * gate) formed in the GEMM's B-operand loads (sm_linear_dw_se): bit-identical to
    se_scale + linear_dw (the same split-K tiles and order), and the fp32 torch math of
    the same bf16 h3.  Shapes: one-frame-per-K-step boundary (HW = 64), ragged channel
    tile (C = 200: columns past N), split-K at the stage-1 / stage-0 step shapes
    (Fr = 64 x 112^2 = 0.8 M rows), a single 8 x 8 tile."""
    kk = KK()
    M = Fr * HW
    a2 = rnd(M, C, dtype=torch.bfloat16, seed=180, scale=2.0).to(DEV)
    dy = rnd(M, N, dtype=torch.bfloat16, seed=181, scale=0.1).to(DEV)
    mean = (torch.randn(C, generator=torch.Generator().manual_seed(182)) * 0.3).to(DEV)
    rstd = (torch.rand(C, generator=torch.Generator().manual_seed(183)) + 0.5).to(DEV)
    w = (torch.rand(C, generator=torch.Generator().manual_seed(184)) + 0.5).to(DEV)
    b = (torch.randn(C, generator=torch.Generator().manual_seed(185)) * 0.1).to(DEV)
    gate = torch.rand(Fr, C, generator=torch.Generator().manual_seed(186)).to(DEV)
    act = (mean, rstd, w, b, True)
    h3 = kk.se_scale(a2, gate, Fr, HW, C, act=act)
    g1 = torch.full((N, C), 0.25, device=DEV)
    g2 = g1.clone()
    kk.linear_dw(dy, h3, g1, accumulate=acc)
    kk.linear_dw_se(dy, a2, act, gate, HW, g2, accumulate=acc)
    assert torch.equal(g1, g2)
    ref = dy.float().t() @ h3.float() + (0.25 if acc else 0.0)
    assert rel_err(g2, ref) < 1e-3
    if Fr <= 5:   # h3 itself against fp32 torch math (bf16 roundings as the kernels)
        hh = F.gelu((a2.float() * (rstd * w) + (b - mean * rstd * w))).to(torch.bfloat16).float()
        hh = (hh.view(Fr, HW, C) * gate.view(Fr, 1, C)).view(M, C)
        assert rel_err(h3.float(), hh) < 1e-2


@pytest.mark.parametrize("case", ["bias", "bias_unaligned", "gelu", "branch", "dx", "dx_res", "k128", "k40",
                                  "stats", "k384", "k384_branch", "dx_k384", "stats_k192", "gelu_aux",
                                  "gelu_aux_k384", "gelu_bwd", "gelu_bwd_k384", "k384_n264",
                                  "dx_k384_n264", "gelu_bwd_noh"])
def test_gemm_persistent_bit_identical(case):
    """The persistent GEMM form (gemm_bf16_pp: tile epilogues written through LDS and stored
    under the next tile's K loop; K <= 128 at 8 tiles per block, K <= 384 with N >= 512 at 2)
    against the one-tile-per-block v2 form, bit for bit: ragged M (a partial last m-tile) and
    N (392 / 520: a partial n-tile), K tails (96, 40: one K-step; 384, 192: several), every
    epilogue option of the plain form (bias, GELU without / with its pre-activation side output,
    the autocast-rounded branch + dropout + DropPath + residual), the data-gradient layout (M/N-major B), the
    BatchNorm-statistics epilogue, and the GELU-backward data gradient with its activation side output
    (sm_linear_dx_gelu, with / without dropout).  > 512 tiles: the persistent path."""
    kk = KK()
    M, N, Kd = 256 * 200 + 77, 392, 96
    if case == "k128":
        Kd = 128
    elif case == "k40":
        Kd = 40
    elif case in ("k384", "k384_branch", "dx_k384", "gelu_aux_k384", "gelu_bwd_k384"):
        N, Kd = 520, 384
    elif case in ("k384_n264", "dx_k384_n264"):   # K = 384 below N = 512 (persistent since round 6)
        N, Kd = 264, 384
    elif case == "stats":
        M, N = 256 * 300 + 13, 384
    elif case == "stats_k192":
        M, N, Kd = 256 * 300 + 13, 768, 192
    x = rnd(M, Kd, dtype=torch.bfloat16, seed=310).to(DEV)
    w = rnd(N, Kd, dtype=torch.bfloat16, seed=311, scale=0.2).to(DEV)
    bias_buf = rnd(N + 1, seed=312).to(DEV)
    bias = bias_buf[1:] if case == "bias_unaligned" else bias_buf[:N]
    res = rnd(M, N, dtype=torch.bfloat16, seed=313).to(DEV)
    rs = (torch.rand(64, generator=torch.Generator().manual_seed(314)) * 2).to(DEV)

    def run():
        if case in ("dx", "dx_res", "dx_k384", "dx_k384_n264"):   # dX[M][Kd'] = dy[M][N] w[N][Kd']: here dy = x, w' = [Kd][N']
            n2 = 520 if case == "dx_k384" else 264
            wt = rnd(Kd, n2, dtype=torch.bfloat16, seed=315, scale=0.2).to(DEV)
            r2 = rnd(M, n2, dtype=torch.bfloat16, seed=316).to(DEV) if case == "dx_res" else None
            return (kk.linear_dx(x, wt, residual=r2),)
        if case in ("stats", "stats_k192"):
            rm, rv = torch.zeros(N, device=DEV), torch.ones(N, device=DEV)
            nb = torch.zeros((), dtype=torch.int64, device=DEV)
            return kk.linear_bn_stats(x, w, rm, rv, 0.1, 1e-5, 1, nb) + (rm, rv)
        if case in ("gelu_bwd", "gelu_bwd_k384", "gelu_bwd_noh"):   # fc2 dX through dropout(GELU(pre)) (+ h)
            wt = rnd(Kd, 520, dtype=torch.bfloat16, seed=317, scale=0.2).to(DEV)
            pre = rnd(M, 520, dtype=torch.bfloat16, seed=318).to(DEV)
            if case == "gelu_bwd_noh":   # without the side output (sm_gemm's IMP 9 path)
                return (kk.linear_dx(x, wt, gelu_pre=pre, drop_p=0.1, seed=80),)
            return kk.linear_dx_gelu(x, wt, pre, 0.1 if case == "gelu_bwd" else 0.0, 79)
        if case in ("gelu_aux", "gelu_aux_k384"):   # fc1: GELU + the pre-activation side output
            drop = 0.1 if case == "gelu_aux" else 0.0
            return kk.linear(x, w, bias, gelu=True, round_branch=True, drop_p=drop, seed=78)
        out = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
        if case == "gelu":
            kk.gemm(x, w, out, M, N, Kd, 0, 0, Kd, Kd, N, bias=bias, gelu=True)
        elif case in ("branch", "k384_branch"):
            kk.gemm(x, w, out, M, N, Kd, 0, 0, Kd, Kd, N, bias=bias, beta=1.0, R=res, round_branch=True,
                    drop_p=0.1, seed=77, row_scale=rs, rows_per_group=M // 63)
        else:
            kk.gemm(x, w, out, M, N, Kd, 0, 0, Kd, Kd, N, bias=bias)
        return (out,)

    prev = kk.gemm_persistent(0)
    try:
        ref = run()
        kk.gemm_persistent(1)
        got = run()
    finally:
        kk.gemm_persistent(prev)
    for a, b in zip(got, ref):
        assert torch.equal(a, b), case
    if case in ("bias", "k384"):
        assert rel_err(got[0], x.float() @ w.float().t() + bias) < TOL[torch.bfloat16]


@pytest.mark.parametrize("M,N,Kd,upd", [(100000, 384, 96, 2), (1000, 384, 96, 1), (100, 96, 64, 1), (4097, 40, 32, 2),
                                        (12544 * 32, 384, 96, 2), (12544 * 32 + 77, 384, 96, 1),
                                        (12544 * 32, 384, 64, 1)])
def test_linear_bn_stats(M, N, Kd, upd):
    """Expand conv + its BatchNorm statistics from the GEMM epilogue (sm_linear_bn_stats):
    y bit-identical to linear(), mean / rstd / running statistics within fp32 rounding of
    bn_stats() over the same stored y (different fixed summation order), and
    num_batches_tracked advanced `upd` times.  Shapes: ragged M (partial tiles and 64-row
    slabs past M), the BM = 128 tile (M < 192), a ragged output width (N = 40); M >= 12544 * 32
    takes the persistent GEMM form (>= 2048 tiles, K <= 128: both linear() and
    linear_bn_stats()), ragged and with one K-step (K = 64), checked against fp32 torch."""
    kk = KK()
    x = rnd(M, Kd, dtype=torch.bfloat16, seed=200).to(DEV)
    w = rnd(N, Kd, dtype=torch.bfloat16, seed=201, scale=0.3).to(DEV)
    rm1, rv1 = torch.full((N,), 0.1, device=DEV), torch.full((N,), 2.0, device=DEV)
    rm2, rv2 = rm1.clone(), rv1.clone()
    nb1 = torch.zeros((), dtype=torch.int64, device=DEV)
    nb2 = nb1.clone()
    y1 = kk.linear(x, w)
    m1, r1 = kk.bn_stats(y1, rm1, rv1, 0.1, 1e-5, upd, nb1)
    y2, m2, r2 = kk.linear_bn_stats(x, w, rm2, rv2, 0.1, 1e-5, upd, nb2)
    assert torch.equal(y1, y2)
    assert rel_err(m2, m1) < 1e-5 and rel_err(r2, r1) < 1e-5
    assert rel_err(rm2, rm1) < 1e-5 and rel_err(rv2, rv1) < 1e-5
    assert int(nb2) == upd == int(nb1)
    yf = y1.float()
    assert rel_err(m2, yf.mean(0)) < 1e-4
    assert rel_err(r2, 1.0 / torch.sqrt(yf.var(0, unbiased=False) + 1e-5)) < 1e-4
    if M >= 100000:
        assert rel_err(y1, x.float() @ w.float().t()) < TOL[torch.bfloat16]


@pytest.mark.parametrize("shape,frames", [((2, 3, 3, 37, 30), False), ((1, 3, 8, 224, 224), False),
                                          ((5, 3, 17, 23), True), ((32, 3, 8, 224, 224), False)])
def test_stem_conv1_direct(shape, frames):
    """Stem conv1 straight from the strided fp32 clip (sm_stem_conv1_bn_stats): a1
    bit-identical to stem_im2col + linear_bn_stats (the same MFMA products and order),
    BN1 statistics / running statistics within fp32 rounding of the GEMM epilogue's.
    Shapes: odd frame sizes (Ho = 19, Wo = 15: pixel segments straddle rows), one full
    clip, a frames view [N,3,H,W] with a non-contiguous layout, B = 32 clips at 224^2."""
    kk = KK()
    g = torch.Generator().manual_seed(220)
    if frames:
        clip = torch.randn(shape[0], shape[2], shape[3], shape[1], generator=g).to(DEV).permute(0, 3, 1, 2)
    else:
        clip = torch.randn(*shape, generator=g).to(DEV)
    wp = kk.conv_wpack((torch.randn(48, 3, 3, 3, generator=g) * 0.2).to(DEV), 32, 0, torch.bfloat16)
    rm1, rv1 = torch.full((48,), 0.1, device=DEV), torch.full((48,), 2.0, device=DEV)
    rm2, rv2 = rm1.clone(), rv1.clone()
    nb1 = torch.zeros((), dtype=torch.int64, device=DEV)
    nb2 = nb1.clone()
    col, geom1 = kk.stem_im2col(clip, torch.bfloat16)
    y1, m1, r1 = kk.linear_bn_stats(col, wp, rm1, rv1, 0.1, 1e-5, 1, nb1)
    y2, m2, r2, geom2 = kk.stem_conv1_bn_stats(clip, wp, rm2, rv2, 0.1, 1e-5, 1, nb2)
    assert geom1 == geom2
    assert torch.equal(y1, y2)
    assert rel_err(m2, m1) < 1e-5 and rel_err(r2, r1) < 1e-5
    assert rel_err(rm2, rm1) < 1e-5 and rel_err(rv2, rv1) < 1e-5
    assert int(nb2) == 1 == int(nb1)


@pytest.mark.parametrize("Fn,H,W,gelu", [(3, 14, 12, True), (2, 9, 23, True), (32, 112, 112, True),
                                         (1, 5, 128, True), (2, 1, 7, False), (3, 3, 33, False),
                                         (2, 7, 110, True), (1, 4, 109, False), (2, 2, 112, True)])
def test_stem_conv2_direct(Fn, H, W, gelu):
    """Stem conv2 over act(a1) with BN1 (+GELU) applied in the kernel's LDS ring
    (sm_stem_conv2_bn_stats): y bit-identical to conv3x3_fwd(bn_apply(a1)) (same k order
    and MFMA chain), BN2 statistics / running statistics within fp32 rounding.  Shapes:
    ragged pixel segments (W = 12, 23, 33), the bench frame (112^2, 32 frames), the widest
    frame (W = 128), a single row (H = 1), odd band counts; identity activation.  W >= 110
    takes the LDS-staged 16-B-store epilogue (W = 110 its smallest frame, 109 the direct form)."""
    kk = KK()
    g = torch.Generator().manual_seed(230)
    a1 = (torch.randn(Fn * H * W, 48, generator=g) * 2).to(torch.bfloat16).to(DEV)
    m1 = (torch.randn(48, generator=g) * 0.3).to(DEV)
    r1 = (torch.rand(48, generator=g) + 0.5).to(DEV)
    g1 = (torch.rand(48, generator=g) + 0.5).to(DEV)
    b1 = (torch.randn(48, generator=g) * 0.1).to(DEV)
    wp = kk.conv_wpack((torch.randn(96, 48, 3, 3, generator=g) * 0.05).to(DEV), 432, 1, torch.bfloat16)
    rm1, rv1 = torch.full((96,), 0.1, device=DEV), torch.full((96,), 2.0, device=DEV)
    rm2, rv2 = rm1.clone(), rv1.clone()
    nb1 = torch.zeros((), dtype=torch.int64, device=DEV)
    nb2 = nb1.clone()
    h1 = kk.bn_apply(a1, m1, r1, g1, b1, gelu=gelu)
    y1, mm1, rr1 = kk.conv3x3_fwd_bn_stats(h1, wp, Fn, H, W, 48, 96, rm1, rv1, 0.1, 1e-5, 1, nb1)
    y2, mm2, rr2 = kk.stem_conv2_bn_stats(a1, (m1, r1, g1, b1, gelu), wp, Fn, H, W, rm2, rv2, 0.1, 1e-5, 1, nb2)
    assert torch.equal(y1, y2)
    assert rel_err(mm2, mm1) < 1e-5 and rel_err(rr2, rr1) < 1e-5
    assert rel_err(rm2, rm1) < 1e-5 and rel_err(rv2, rv1) < 1e-5
    assert int(nb2) == 1 == int(nb1)


@pytest.mark.parametrize("Fn,H,W,Cin,Cout,upd", [(3, 14, 12, 48, 96, 1), (2, 9, 23, 16, 24, 2),
                                                  (32, 112, 112, 48, 96, 1), (1, 3, 5, 8, 8, 1)])
def test_conv3x3_fwd_bn_stats(Fn, H, W, Cin, Cout, upd):
    """Stem conv2 + BN2 statistics from the implicit-conv GEMM's epilogue
    (sm_conv3x3_fwd_bn_stats): y bit-identical to conv3x3_fwd, statistics / running
    statistics within fp32 rounding of bn_stats over the same y.  Shapes: ragged pixel
    tiles and 64-row slabs, the B = 8 clip frame count at 112^2 (32 frames), 15 pixels."""
    kk = KK()
    x = rnd(Fn * H * W, Cin, dtype=torch.bfloat16, seed=210).to(DEV)
    wp = kk.conv_wpack(rnd(Cout, Cin, 3, 3, seed=211).to(DEV) * 0.1, 9 * Cin, 1, torch.bfloat16)
    rm1, rv1 = torch.full((Cout,), 0.1, device=DEV), torch.full((Cout,), 2.0, device=DEV)
    rm2, rv2 = rm1.clone(), rv1.clone()
    nb1 = torch.zeros((), dtype=torch.int64, device=DEV)
    nb2 = nb1.clone()
    y1 = kk.conv3x3_fwd(x, wp, Fn, H, W, Cin, Cout)
    m1, r1 = kk.bn_stats(y1, rm1, rv1, 0.1, 1e-5, upd, nb1)
    y2, m2, r2 = kk.conv3x3_fwd_bn_stats(x, wp, Fn, H, W, Cin, Cout, rm2, rv2, 0.1, 1e-5, upd, nb2)
    assert torch.equal(y1, y2)
    assert rel_err(m2, m1) < 1e-5 and rel_err(r2, r1) < 1e-5
    assert rel_err(rm2, rm1) < 1e-5 and rel_err(rv2, rv1) < 1e-5
    assert int(nb2) == upd == int(nb1)


@pytest.mark.parametrize("Fr,HW,N,C", [(3, 128, 96, 384), (2, 256, 192, 768), (16, 12544, 96, 384),
                                       (5, 384, 40, 64), (1, 128, 8, 1536)])
def test_linear_se_operand(Fr, HW, N, C):
    """MBConv projection forward over the SE output with h3 = bf16(bf16(GELU(BN(a2))) *
    gate) formed in the GEMM's A-operand loads (sm_linear_se): bit-identical to se_fwd's
    h3 + linear, and the gate-only SE call (se_fwd, y = null) returns the same pooled /
    hidden / gate.  Shapes: tiles of one frame at HW = 128, the stage-0 frame (112^2),
    a ragged output width (N = 40: columns past N), K = 64 and K = 1536 (the table bound)."""
    kk = KK()
    M = Fr * HW
    a2 = rnd(M, C, dtype=torch.bfloat16, seed=190, scale=2.0).to(DEV)
    w = rnd(N, C, dtype=torch.bfloat16, seed=191, scale=0.1).to(DEV)
    mean = (torch.randn(C, generator=torch.Generator().manual_seed(192)) * 0.3).to(DEV)
    rstd = (torch.rand(C, generator=torch.Generator().manual_seed(193)) + 0.5).to(DEV)
    gw = (torch.rand(C, generator=torch.Generator().manual_seed(194)) + 0.5).to(DEV)
    gb = (torch.randn(C, generator=torch.Generator().manual_seed(195)) * 0.1).to(DEV)
    act = (mean, rstd, gw, gb, True)
    R = C // 4
    w1 = rnd(R, C, seed=196, scale=0.1).to(DEV)
    w2 = rnd(C, R, seed=197, scale=0.1).to(DEV)
    h3, pooled, h1, gate = kk.se_fwd(a2, Fr, HW, C, w1, w2, act=act)
    y_none, pooled2, h12, gate2 = kk.se_fwd(a2, Fr, HW, C, w1, w2, act=act, want_y=False)
    assert y_none is None and torch.equal(pooled, pooled2) and torch.equal(h1, h12) and torch.equal(gate, gate2)
    ref = kk.linear(h3, w)
    y = kk.linear_se(a2, w, act, gate, HW)
    assert y.dtype == torch.bfloat16 and torch.equal(y, ref)
    assert rel_err(y.float(), h3.float() @ w.float().t()) < 1e-2


@pytest.mark.parametrize("Fr,H,C,s", [(4, 19, 64, 2), (4, 20, 64, 2), (3, 30, 32, 2), (2, 56, 768, 2),
                                      (4, 7, 1536, 2), (4, 4, 768, 2), (4, 8, 384, 2),
                                      (4, 19, 64, 1), (2, 112, 96, 1)])
def test_dwconv_bn_bwd_vs_fp32(Fr, H, C, s):
    """The fused depthwise + BatchNorm0/GELU backward (sm_dwconv_bn_bwd, stride 1;
    sm_dwconv_s2_bn_bwd, stride 2: odd and even sizes, ragged last strips, the zero
    dy row past Ho) against fp32 autograd of conv2d(GELU(batch_norm(x)), groups=C) from
    the same bf16 inputs, and against the unfused sequence (depthwise backward, then
    bn_bwd)."""
    kk = KK()
    W = H
    Ho = (H - 1) // s + 1
    a1 = (rnd(Fr * H * W, C, seed=180, scale=1.5) + 0.2).to(torch.bfloat16).to(DEV)
    g0 = (rnd(C, seed=181, scale=0.2) + 1.0).to(DEV)
    b0 = rnd(C, seed=182, scale=0.2).to(DEV)
    wdw = rnd(C, 9, seed=183, scale=0.3).to(DEV)
    m0, r0 = kk.bn_stats(a1)
    act0 = (m0, r0, g0, b0, True)
    da2 = rnd(Fr * Ho * Ho, C, dtype=torch.bfloat16, seed=184, scale=1e-2).to(DEV)
    dw_f = torch.zeros(C, 9, device=DEV)
    dg_f, db_f = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
    da1 = kk.dwconv_bn_bwd(da2, a1, act0, wdw, dw_f, dg_f, db_f, Fr, H, W, C, stride=s)
    dw_u = torch.zeros(C, 9, device=DEV)
    dh1 = kk.dwconv_fused_bwd(da2, a1, act0, wdw, dw_u, Fr, H, W, C, s)
    dg_u, db_u = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
    da1_u = kk.bn_bwd(dh1, a1, m0, r0, g0, b0, True, dg_u, db_u)
    x = a1.float().view(Fr, H, W, C).permute(0, 3, 1, 2).contiguous().requires_grad_(True)
    tg, tb, tw = g0.clone().requires_grad_(True), b0.clone().requires_grad_(True), wdw.clone().requires_grad_(True)
    y = F.conv2d(F.gelu(F.batch_norm(x, None, None, tg, tb, True, 0.0, 1e-5)), tw.view(C, 1, 3, 3), None, s, 1, 1, C)
    y.backward(da2.float().view(Fr, Ho, Ho, C).permute(0, 3, 1, 2))
    gx = x.grad.permute(0, 2, 3, 1).reshape(-1, C)
    assert rel_err(da1, gx) < 2e-2 and rel_err(da1, da1_u) < 2e-2
    assert rel_err(dw_f, tw.grad) < 1e-2 and rel_err(dw_f, dw_u) < 1e-2
    assert rel_err(dg_f, tg.grad) < 2e-2 and rel_err(db_f, tb.grad) < 2e-2


@pytest.mark.parametrize("Kd,N", [(96, 392), (384, 520)])
def test_gemm_persistent_ragged_operands_at_allocation_end(Kd, N):
    """gemm_bf16_pp with a ragged last m-tile (M % 256 = 77) and a ragged last n-tile whose A and
    B rows end exactly at the end of their allocations (views onto the tail of a 2-MiB-multiple
    buffer): every chunk's row is range-checked through its VGPR offset, so rows past M / N
    read zero instead of memory past the allocation (the scalar-offset form left
    chunks 1-3 of the last tile unchecked).  Bit-identical to the one-tile-per-block form."""
    kk = KK()
    M = 256 * 40 + 77

    def tail_view(rows, cols, seed):
        n = rows * cols
        cap = ((n * 2 + (2 << 20) - 1) // (2 << 20)) * (2 << 20) // 2
        buf = torch.empty(cap, dtype=torch.bfloat16, device=DEV)
        v = buf[cap - n:].view(rows, cols)
        v.copy_(rnd(rows, cols, dtype=torch.bfloat16, seed=seed).to(DEV))
        return v

    x = tail_view(M, Kd, 401)
    w = tail_view(N, Kd, 402)
    outs = []
    prev = kk.gemm_persistent(0)
    try:
        for mode in (0, 1):
            kk.gemm_persistent(mode)
            out = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
            kk.gemm(x, w, out, M, N, Kd, 0, 0, Kd, Kd, N)
            outs.append(out)
    finally:
        kk.gemm_persistent(prev)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    assert rel_err(outs[1], x.float() @ w.float().t()) < TOL[torch.bfloat16]
