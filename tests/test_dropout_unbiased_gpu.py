"""Every dropout / DropPath site of the step is unbiased: E[mask * scale] = 1, as the
reference's nn.Dropout (nn.TransformerEncoderLayer's four dropout sites per decoder layer,
/root/reference/src/models/mae_vit_adapter.py:39-47) and timm DropPath
(/root/reference/src/models/tiny_vit.py:52,114).

The keep decision is the counter hash's quantised threshold (8-bit round(256 p) for the
GEMM / elementwise / DropPath sites, 7-bit round(128 p) for the attention probabilities),
so the kernels scale kept values by the inverse of that quantised keep rate:
256 / (256 - thr) and 128 / (128 - thr).  Per site the test recovers mask * scale
elementwise from the kernel's own outputs (with / without dropout on the same inputs),
checks that it takes exactly the two values {0, scale}, and that its empirical mean is 1
within 4 standard errors (n >= 1.5 M draws: sigma ~ 2.7e-4; the old 1 / (1 - p) scale sat
1.7e-3 low, > 6 sigma).
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"
P = 0.1


@pytest.fixture(scope="module", autouse=True)
def _lib():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from ssl_mae_amd import _lib as L
    L.load()


def KK():
    from ssl_mae_amd import kernels
    return kernels


def _scale(p, q):
    return q / (q - int(p * q + 0.5))


def _check(ms, scale):
    """ms: samples of mask * scale (float64, flat)."""
    ms = ms.double().flatten()
    zero = ms == 0
    assert torch.allclose(ms[~zero], torch.full_like(ms[~zero], scale), rtol=2e-6, atol=0), \
        f"kept values not scaled by {scale}"
    n = ms.numel()
    keep = 1.0 - zero.double().mean().item()
    sigma = scale * math.sqrt(keep * (1 - keep) / n)
    mean = ms.mean().item()
    assert abs(mean - 1.0) < 4 * sigma + 1e-12, f"E[mask*scale] = {mean:.6f} (sigma {sigma:.2e}, n {n})"
    return mean


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_gemm_epilogue_dropout_unbiased(dtype):
    """Decoder FF / residual dropout in the GEMM epilogue (linear(..., drop_p))."""
    kk = KK()
    M, N, Kd = 4096, 384, 64
    g = torch.Generator(device=DEV).manual_seed(5)
    x = (torch.rand(M, Kd, generator=g, device=DEV) + 0.5).to(dtype)   # positive: no zero products
    w = (torch.rand(N, Kd, generator=g, device=DEV) + 0.5).to(dtype)
    R = torch.zeros(M, N, dtype=torch.float32, device=DEV)
    y0 = kk.linear(x, w, out_dtype=torch.float32, residual=R)
    y = kk.linear(x, w, out_dtype=torch.float32, residual=R, drop_p=P, seed=77)
    _check(y.double() / y0.double(), _scale(P, 256))


def test_elementwise_dropout_unbiased():
    """GELU(+dropout) forward, the dropout backward and the fused cast + dropout backward."""
    kk = KK()
    M, N = 4096, 384
    ones32 = torch.ones(M, N, dtype=torch.float32, device=DEV)
    _check(kk.dropout_bwd(ones32, P, 31), _scale(P, 256))
    cb = kk.cast_dropout_bwd(ones32, P, 32).float().double()           # bf16 out: kept = bf16(scale)
    assert set(torch.unique(cb).tolist()) <= {0.0, float(torch.tensor(_scale(P, 256), dtype=torch.bfloat16))}
    _check((cb != 0).double() * _scale(P, 256), _scale(P, 256))
    g = torch.Generator(device=DEV).manual_seed(6)
    pre = (torch.rand(M, N, generator=g, device=DEV) + 1.0)           # GELU(x) ~ x: no zeros
    h = kk.gelu(pre, P, 33).double()
    h0 = kk.gelu(pre).double()
    _check(h / h0, _scale(P, 256))


def test_droppath_unbiased():
    """DropPath per-sample scale (residual branches of MBConv / TinyViTBlock)."""
    kk = KK()
    _check(kk.droppath_scale(1 << 21, P, 7, DEV), _scale(P, 256))


def test_layernorm_branch_dropout_unbiased():
    """The decoder residual dropout's backward applied by the LayerNorm backward's branch copy."""
    kk = KK()
    M, C = 4096, 384
    x = torch.randn(M, C, device=DEV)
    gam = torch.ones(C, device=DEV)
    bet = torch.zeros(C, device=DEV)
    dy = torch.zeros(M, C, dtype=torch.bfloat16, device=DEV)
    res = torch.ones(M, C, device=DEV)                  # dx = dres = 1 everywhere (dy = 0)
    _, mean, rstd = kk.layernorm(x, gam, bet, out_dtype=torch.bfloat16)
    dg, db = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
    _, dxb = kk.layernorm_bwd_branch(dy, x, mean, rstd, gam, dg, db, dres=res, drop_p=P, seed=41)
    s = _scale(P, 256)
    got = dxb.float().double()
    # the branch copy is bf16: kept values are bf16(s)
    sb = float(torch.tensor(s, dtype=torch.bfloat16))
    assert set(torch.unique(got).tolist()) <= {0.0, sb}
    _check((got != 0).double() * s, s)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_attention_probability_dropout_unbiased(dtype):
    """Attention-probability dropout: with Q = K = 0 every probability is 1/L, and with
    V = 1 each output element is (kept keys of the row) * scale / L; the host regenerates
    the keep count (test_kernels_gpu._np_keep rule), so O * L / count recovers the kernel's
    scale per row (bf16 output: to 2^-9 per row, averaged over rows)."""
    import numpy as np
    from test_kernels_gpu import _np_keep
    kk = KK()
    N, L, H, D, seed = 4, 1024, 6, 64, 2024
    qkv = torch.zeros(N, L, 3, H, D, dtype=dtype)
    qkv[:, :, 2] = 1.0
    qkv = qkv.reshape(N * L, 3 * H * D).to(DEV)
    o, _ = kk.attn_fwd(qkv, N, L, H, D, drop_p=P, seed=seed)
    o = o.float().reshape(N, L, H, D)[..., 0].permute(0, 2, 1).reshape(-1).double().cpu()   # [(n, h, q)]
    keep = _np_keep(np.arange(N * H * L), np.arange(L), P, seed, attn=True)
    count = torch.from_numpy(keep.sum(1).astype(np.float64))
    s = _scale(P, 128)
    est = (o * L / count)
    if dtype == torch.float32:
        assert torch.allclose(est, torch.full_like(est, s), rtol=1e-5)
    else:
        assert abs(est.mean().item() - s) < 2e-4
    _check(torch.from_numpy(keep.astype(np.float64)).flatten() * s, s)
