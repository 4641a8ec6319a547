"""The bf16 GEMM's K loop on v_mfma_f32_16x16x32_bf16 (csrc/gemm.hip: gemm_bf16_v2 MF = 16,
mma16_col + acc16_to_32), selected by sm_gemm_tuning key mf16_min_k for K-major-A tiles.

Reference ops: the Linear layers of the reference model (nn.Linear forward x @ W^T + b and its
autograd data gradient dy @ W; /root/reference/src/models/mae_vit_adapter.py,
tiny_vit.py).  Each case runs with the 16x16x32 loop forced on, against torch fp32 math on
the same bf16 operands (max-abs error relative to the output's max: 1e-2 for bf16 outputs,
1e-4 for fp32 outputs), and against the default 32x32x16 loop (the products are exact in
fp32, only the accumulation order differs: fp32 outputs within 1e-5 relative, bf16 outputs
within one bf16 rounding step, 2^-7 relative).  Ragged M / N / K, split-K (k_chunk < K),
the GELU / residual / bias epilogues, both B layouts and both output types.
"""
import contextlib

import pytest
import torch

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


@contextlib.contextmanager
def mf16(on):
    kk = KK()
    prev = kk.gemm_tuning("mf16_min_k", 0 if on else 1 << 30)
    try:
        yield
    finally:
        kk.gemm_tuning("mf16_min_k", prev)


def rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).abs().max() / (b.abs().max() + 1e-12)).item()


def _operands(M, N, K, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    x = torch.randn(M, K, generator=g, device=DEV).to(torch.bfloat16)
    w = (torch.randn(N, K, generator=g, device=DEV) * K ** -0.5).to(torch.bfloat16)
    b = torch.randn(N, generator=g, device=DEV)
    dy = torch.randn(M, N, generator=g, device=DEV).to(torch.bfloat16)
    return x, w, b, dy


@pytest.mark.parametrize("M,N,K", [(1000, 200, 1536), (777, 1152, 384), (2048, 384, 200), (300, 96, 72),
                                   (256, 256, 8192)])
@pytest.mark.parametrize("out", [torch.bfloat16, torch.float32])
def test_linear_fwd_mf16(M, N, K, out):
    kk = KK()
    x, w, b, _ = _operands(M, N, K, M + N + K)
    ref = x.float() @ w.float().t() + b
    with mf16(True):
        y16 = kk.linear(x, w, b, out_dtype=out)
    with mf16(False):
        y32 = kk.linear(x, w, b, out_dtype=out)
    assert rel(y16, ref) < (1e-2 if out == torch.bfloat16 else 1e-4)
    assert rel(y16, y32) < (2 ** -7 if out == torch.bfloat16 else 1e-5)


@pytest.mark.parametrize("M,N,K", [(1000, 1536, 384), (513, 384, 1152), (4096, 200, 96)])
@pytest.mark.parametrize("out", [torch.bfloat16, torch.float32])
def test_linear_dx_mf16(M, N, K, out):
    """dx = dy @ w: A = dy K-major, B = w stored [K = N_out][N_in] (M/N-major tile, transposed reads)."""
    kk = KK()
    _, w, _, dy = _operands(M, N, K, 3 * M + N)
    ref = dy.float() @ w.float()
    with mf16(True):
        d16 = kk.linear_dx(dy, w, out_dtype=out)
    with mf16(False):
        d32 = kk.linear_dx(dy, w, out_dtype=out)
    assert rel(d16, ref) < (1e-2 if out == torch.bfloat16 else 1e-4)
    assert rel(d16, d32) < (2 ** -7 if out == torch.bfloat16 else 1e-5)


def test_linear_gelu_residual_mf16():
    """fc1-style GELU epilogue with its pre-activation side output, and a residual add."""
    kk = KK()
    M, N, K = 1500, 1536, 384
    x, w, b, _ = _operands(M, N, K, 11)
    R = torch.randn(M, N, device=DEV)
    pre_ref = x.float() @ w.float().t() + b
    with mf16(True):
        h, pre = kk.linear(x, w, b, gelu=True)
        y = kk.linear(x, w, b, out_dtype=torch.float32, residual=R)
    assert rel(pre, pre_ref) < 1e-2
    assert rel(h, torch.nn.functional.gelu(pre_ref)) < 1e-2
    assert rel(y, pre_ref + R) < 1e-4


def test_mf16_threshold_default_off():
    """The product default keeps the 32x32x16 loop until a measured threshold is set."""
    kk = KK()
    v = kk.gemm_tuning("mf16_min_k")
    assert v >= 384 or v == 1 << 30
