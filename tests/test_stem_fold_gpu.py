"""The stem's BN2 folded into stage 0's first MBConv (reference
tiny_vit.py:62-72 PatchEmbed -> :36-56 MBConv, stages[0][0]).

PatchEmbed's last BatchNorm output y = BN2(a2) has one consumer, stages[0][0].  With the
fold, y is never written: the expand conv's A operand, the residual add and the expand
weight gradient's B operand each form bf16(a2 sc + sh) in their own loads, exactly as
bn_apply stores y.  These tests pin that equivalence BIT FOR BIT:
  * kernel level: sm_linear_bnin(_bn_stats), sm_bn_apply_res_bn and sm_linear_dw_se with
    no gate against bn_apply followed by the unfused kernel, at the stage-0 shape class
    (K = 96 channels, N = 384) and ragged shapes;
  * model level: two bf16 training steps (dropout / DropPath on) with the fold on and off
    give identical losses, parameters after AdamW and BatchNorm buffers, for each stage-0
    memory policy (resident, lite-resident, checkpointed).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from ssl_mae_amd import _lib
    _lib.load()


def KK():
    from ssl_mae_amd import kernels
    return kernels


def _bn(C, seed):
    g = torch.Generator().manual_seed(seed)
    mean = (torch.randn(C, generator=g) * 0.3).to(DEV)
    rstd = (torch.rand(C, generator=g) + 0.5).to(DEV)
    w = (torch.rand(C, generator=g) + 0.5).to(DEV)
    b = (torch.randn(C, generator=g) * 0.1).to(DEV)
    return mean, rstd, w, b


def _rnd(*shape, seed, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(torch.bfloat16).to(DEV)


@pytest.mark.parametrize("M,N,K", [(2 * 12544, 384, 96), (1000, 384, 96), (300, 40, 24), (130, 136, 256),
                                   (48 * 12544 + 77, 384, 96), (256 * 300 + 13, 520, 192)])
def test_linear_bnin_bit_identical(M, N, K):
    """(the last two: > 512 tiles -- the persistent GEMM form, ragged M; K = 96 at 8 tiles per block,
    K = 192 with N >= 512 at 2)"""
    kk = KK()
    a = _rnd(M, K, seed=1, scale=2.0)
    w = _rnd(N, K, seed=2, scale=0.2)
    mean, rstd, bw, bb = _bn(K, 3)
    y_ref = kk.bn_apply(a, mean, rstd, bw, bb, gelu=False)
    ref = kk.linear(y_ref, w)
    got = kk.linear_bnin(a, (mean, rstd, bw, bb, False), w)
    assert got.dtype == torch.bfloat16 and torch.equal(got, ref)
    # + the output's BatchNorm statistics: = linear_bn_stats over the stored y
    rm1, rv1 = torch.full((N,), 0.1, device=DEV), torch.full((N,), 2.0, device=DEV)
    rm2, rv2 = rm1.clone(), rv1.clone()
    nb1 = torch.zeros((), dtype=torch.int64, device=DEV)
    nb2 = nb1.clone()
    y1, m1, r1 = kk.linear_bn_stats(y_ref, w, rm1, rv1, 0.1, 1e-5, 2, nb1)
    y2, m2, r2 = kk.linear_bnin(a, (mean, rstd, bw, bb, False), w, (rm2, rv2, 0.1, 1e-5, nb2), 2)
    assert torch.equal(y1, y2) and torch.equal(m1, m2) and torch.equal(r1, r2)
    assert torch.equal(rm1, rm2) and torch.equal(rv1, rv2) and int(nb1) == int(nb2) == 2


@pytest.mark.parametrize("M,C,rows_per_group", [(2 * 12544, 96, 12544), (777, 96, 1), (64, 8, 8)])
def test_bn_apply_residual_bn_bit_identical(M, C, rows_per_group):
    kk = KK()
    a3 = _rnd(M, C, seed=4)
    a2 = _rnd(M, C, seed=5, scale=2.0)
    m5, r5, w5, b5 = _bn(C, 6)
    xbn = _bn(C, 7)
    rs = (torch.rand(max(1, M // rows_per_group), generator=torch.Generator().manual_seed(8)) * 2).to(DEV)
    x = kk.bn_apply(a2, *xbn, gelu=False)
    ref = kk.bn_apply(a3, m5, r5, w5, b5, residual=x, row_scale=rs, rows_per_group=rows_per_group)
    got = kk.bn_apply(a3, m5, r5, w5, b5, residual=a2, row_scale=rs, rows_per_group=rows_per_group,
                      residual_bn=xbn)
    assert torch.equal(got, ref)


@pytest.mark.parametrize("rows,nout,nin", [(2 * 12544, 384, 96), (1000, 384, 96), (4100, 40, 24)])
def test_linear_dw_bn_operand_bit_identical(rows, nout, nin):
    kk = KK()
    a2 = _rnd(rows, nin, seed=9, scale=2.0)
    dy = _rnd(rows, nout, seed=10, scale=0.1)
    xbn = _bn(nin, 11)
    x = kk.bn_apply(a2, *xbn, gelu=False)
    g1 = torch.full((nout, nin), 0.25, device=DEV)
    g2 = g1.clone()
    kk.linear_dw(dy, x, g1)
    kk.linear_dw_se(dy, a2, xbn + (False,), None, 0, g2)
    assert torch.equal(g1, g2)


def _cfg(B, T, S):
    return {"dataset": {"clip_len": T, "image_size": S, "stride": 4, "train_split": "-"},
            "model": {"decoder_embed_dim": 384, "decoder_depth": 2, "decoder_num_heads": 6},
            "ssl": {"mask_ratio": 0.75, "norm_pix_loss": True},
            "training": {"batch_size": B, "lr": 5e-4, "log_interval": 20}}


def _run(policy, fold, steps=2):
    from ssl_mae_amd.init_rule import apply_rule, synthetic_clip
    from ssl_mae_amd.mae_vit_adapter import TinyVideoMAE
    from ssl_mae_amd.optim import FusedAdamW, GradScaler
    from ssl_mae_amd.tiny_vit import PatchEmbed, tiny_vit_21m_variant
    B, T, S = 2, 2, 64
    cfg = _cfg(B, T, S)
    torch.manual_seed(42)
    enc = tiny_vit_21m_variant(img_size=S)
    enc.resident_stages = (0, 1, 2) if policy == "resident" else (1, 2)
    enc.lite_stages = (0,) if policy == "lite" else ()
    model = TinyVideoMAE(enc, cfg)
    apply_rule(model)
    model = model.to(DEV).train()
    opt = FusedAdamW(model.parameters(), lr=5e-4, weight_decay=0.05)
    clip = torch.from_numpy(synthetic_clip(B, T, S, seed=5)).to(DEV)
    old = PatchEmbed.fold_bn2
    PatchEmbed.fold_bn2 = fold
    try:
        from ssl_mae_amd.train_ssl_mae import train_step
        torch.manual_seed(7)
        losses = [train_step(model, clip, opt, GradScaler(), cfg["ssl"], bf16=True)[0].item() for _ in range(steps)]
    finally:
        PatchEmbed.fold_bn2 = old
    state = {k: v.detach().clone() for k, v in model.state_dict().items()}
    return losses, state


@pytest.mark.parametrize("policy", ["resident", "lite", "checkpoint"])
def test_model_step_fold_on_off_bit_identical(policy):
    l_on, s_on = _run(policy, True)
    l_off, s_off = _run(policy, False)
    assert l_on == l_off, (l_on, l_off)
    assert set(s_on) == set(s_off)
    for k in s_on:
        assert torch.equal(s_on[k], s_off[k]), k
    assert int(s_on["encoder.patch_embed.patch_embed.2.bn.num_batches_tracked"]) == 2
