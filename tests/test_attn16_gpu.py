"""The bf16 attention backward on both MFMA shapes (csrc/attention.hip: attn_bwd_dq_bf16 /
attn_bwd_dkdv_bf16 on v_mfma_f32_32x32x16_bf16, attn_bwd_dq16_bf16 / attn_bwd_dkdv16_bf16 on
v_mfma_f32_16x16x32_bf16), selected per head dim with sm_attn_tuning.

Reference op: F.scaled_dot_product_attention (TinyViT Attention, /root/reference/src/models/
tiny_vit.py:96-106, head dim 32) and nn.MultiheadAttention with dropout 0.1 on the
probabilities (/root/reference/src/models/mae_vit_adapter.py:39-47, head dim 64).
Each shape is checked against fp32 torch math on the same bf16 inputs (ragged L, both head
dims, dropout through the host-regenerated keep mask), and the two shapes against each other
(same inputs: the products differ only in the MFMA's accumulation order).
Tolerances: bf16 outputs, max-abs error relative to the reference's max (3e-2, as
test_kernels_gpu's attention tests); shape vs shape 1e-2.
"""
import contextlib
import math

import numpy as np
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
def bwd_shape(D, shape):
    kk = KK()
    prev = kk.attn_tuning(D, shape)
    try:
        yield
    finally:
        kk.attn_tuning(D, prev)


def rel_err(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return ((a - b).abs().max() / (b.abs().max() + 1e-12)).item()


def _inputs(N, L, H, D, seed):
    g = torch.Generator().manual_seed(seed)
    qkv = (torch.randn(N * L, 3 * H * D, generator=g) * 0.7).to(torch.bfloat16)
    dO = torch.randn(N * L, H * D, generator=g).to(torch.bfloat16)
    return qkv, dO


def _ref(qkv, dO, N, L, H, D, p, seed):
    from test_kernels_gpu import _np_keep
    q, k, v = [t.detach().clone().requires_grad_(True)
               for t in qkv.float().reshape(N, L, 3, H, D).permute(2, 0, 3, 1, 4)]
    P = torch.softmax((q @ k.transpose(-1, -2)) / math.sqrt(D), -1)
    if p > 0:
        keep = torch.from_numpy(_np_keep(np.arange(N * H * L), np.arange(L), p, seed, attn=True)).reshape(N, H, L, L)
        P = P * keep * (128 / (128 - int(p * 128 + 0.5)))
    o = (P @ v).transpose(1, 2).reshape(N * L, H * D)
    o.backward(dO.float())
    return o.detach(), torch.stack([q.grad, k.grad, v.grad]).permute(1, 3, 0, 2, 4).reshape(N * L, 3 * H * D)


@pytest.mark.parametrize("shape", [16, 32])
@pytest.mark.parametrize("D,L,p", [(64, 200, 0.0), (64, 200, 0.1), (64, 129, 0.1), (64, 64, 0.0), (64, 33, 0.1),
                                   (32, 130, 0.0), (32, 784, 0.0), (32, 50, 0.0), (32, 97, 0.1)])
def test_attn_bwd_shape_vs_fp32(shape, D, L, p):
    N, H, seed = 2, 3, 13579
    qkv, dO = _inputs(N, L, H, D, 100 + L + D)
    o_ref, dqkv_ref = _ref(qkv, dO, N, L, H, D, p, seed)
    kk = KK()
    o, lse = kk.attn_fwd(qkv.to(DEV), N, L, H, D, drop_p=p, seed=seed)
    assert rel_err(o, o_ref) < 2e-2
    with bwd_shape(D, shape):
        dqkv = kk.attn_bwd(qkv.to(DEV), o, dO.to(DEV), lse, N, L, H, D, p, seed)
    assert torch.isfinite(dqkv.float()).all()
    for part in range(3):   # dQ, dK, dV separately (each relative to its own scale)
        sl = dqkv.view(N * L, 3, H * D)[:, part]
        rf = dqkv_ref.view(N * L, 3, H * D)[:, part]
        assert rel_err(sl, rf) < 3e-2, ("dq", "dk", "dv")[part]


@pytest.mark.parametrize("D,N,L,H,p", [(64, 2, 6272, 6, 0.1), (32, 8, 3136, 6, 0.0), (32, 16, 784, 12, 0.0)])
def test_attn_bwd_shapes_agree_at_step_lengths(D, N, L, H, p):
    """The two MFMA shapes at the step's sequence lengths (decoder L = 6272 with dropout,
    encoder L = 3136 / 784): the same inputs give gradients within 1e-2 of each other."""
    kk = KK()
    qkv, dO = _inputs(N, L, H, D, 7 + D)
    qkv, dO = qkv.to(DEV), dO.to(DEV)
    o, lse = kk.attn_fwd(qkv, N, L, H, D, drop_p=p, seed=99)
    out = {}
    for shape in (32, 16):
        with bwd_shape(D, shape):
            out[shape] = kk.attn_bwd(qkv, o, dO, lse, N, L, H, D, p, 99).float()
    for part in range(3):
        a = out[16].view(N * L, 3, H * D)[:, part]
        b = out[32].view(N * L, 3, H * D)[:, part]
        assert rel_err(a, b) < 1e-2, ("dq", "dk", "dv")[part]


def test_attn_tuning_switch():
    kk = KK()
    prev = kk.attn_tuning(64)
    assert prev in (16, 32)
    assert kk.attn_tuning(64, 16) == prev
    assert kk.attn_tuning(64) == 16
    kk.attn_tuning(64, prev)
    with pytest.raises(Exception):
        kk.attn_tuning(64, 24)
