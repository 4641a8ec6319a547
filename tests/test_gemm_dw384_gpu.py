"""The 384 x 128 pipelined weight-gradient GEMM (csrc/gemm.hip: gemm_dw384, sm_gemm_tuning key
dw384) against the v2 tiles it replaces.

Reference op: the weight and bias gradients of the reference's Linear layers (autograd of
nn.Linear, /root/reference/src/models/mae_vit_adapter.py:40-48, tiny_vit.py:74-84).  Within a
split both kernels accumulate every output element over the same K order with the same MFMA (at
equal split counts dW was bit-identical, profiles/r06zjk_dw384_ab.txt); the new tile takes its own
split count (whole rounds of one block per CU), so the fp32 partial sums group differently: dW and
the fused bias gradient within 1e-5 relative of v2, and both within 1e-3 of fp32 torch math.  Shapes: the step's
dW shapes that divide the tile (nout x nin = 1536 x 384, 384 x 1536 through the transposed form,
1152 x 384, 384 x 384), a ragged token count (K tail inside the last split) and accumulate on.
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
def dw384(on):
    kk = KK()
    prev = kk.gemm_tuning("dw384", 1 if on else 0)
    try:
        yield
    finally:
        kk.gemm_tuning("dw384", prev)


def rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).abs().max() / (b.abs().max() + 1e-12)).item()


@pytest.mark.parametrize("rows,nout,nin,notr", [(100000, 1536, 384, 0), (100003, 384, 1536, 0), (100003, 384, 1536, 1),
                                                (65536, 1152, 384, 0), (99999, 384, 384, 0)])
@pytest.mark.parametrize("acc", [False, True])
def test_dw384_vs_v2(rows, nout, nin, notr, acc):
    """notr = 1: fc2's [384][1536] gradient kept untransposed on the new tile (fused bias gradient)
    instead of the transposed form with its separate column sums."""
    kk = KK()
    prev_notr = kk.gemm_tuning("dw384_notr", notr)
    g = torch.Generator(device=DEV).manual_seed(rows + nout + nin)
    dy = (torch.randn(rows, nout, generator=g, device=DEV) * 0.1).to(torch.bfloat16)
    x = torch.randn(rows, nin, generator=g, device=DEV).to(torch.bfloat16)
    base_w = torch.randn(nout, nin, generator=g, device=DEV) if acc else torch.zeros(nout, nin, device=DEV)
    base_b = torch.randn(nout, generator=g, device=DEV) if acc else torch.zeros(nout, device=DEV)
    out = {}
    try:
        for on in (False, True):
            gw, gb = base_w.clone(), base_b.clone()
            with dw384(on):
                kk.linear_dw_bias(dy, x, gw, gb)
            out[on] = (gw, gb)
    finally:
        kk.gemm_tuning("dw384_notr", prev_notr)
    assert rel(out[True][0], out[False][0]) < 1e-5
    assert rel(out[True][1], out[False][1]) < 1e-5
    ref_w = base_w + dy.float().t() @ x.float()
    ref_b = base_b + dy.float().sum(0)
    assert rel(out[True][0], ref_w) < 1e-3
    assert rel(out[True][1], ref_b) < 1e-3
