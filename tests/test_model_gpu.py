"""End-to-end parity of the HIP training step against the reference.

fp32 mode (no autocast) must match the golden fixtures produced by running the
reference itself (tests/golden/make_golden.py) within 1e-3 (north star); the tube
mask must be bit-exact.  bf16 mode (autocast, the benchmarked path) is compared
with the CPU oracle at bf16-appropriate tolerances (stated per assertion).
"""
import math
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _cfg(B, T, S, ratio, dec_depth=4):
    return {"dataset": {"clip_len": T, "image_size": S, "stride": 4, "train_split": "-"},
            "model": {"decoder_embed_dim": 384, "decoder_depth": dec_depth, "decoder_num_heads": 6},
            "ssl": {"mask_ratio": ratio, "norm_pix_loss": True},
            "training": {"batch_size": B, "lr": 5e-4, "log_interval": 20}}


def _build(cfg, small=False):
    from ssl_mae_amd.init_rule import apply_rule
    from ssl_mae_amd.mae_vit_adapter import TinyVideoMAE
    from ssl_mae_amd.tiny_vit import tiny_vit_21m_variant, tiny_vit_small_variant
    from ssl_mae_amd import parity_mode
    make = tiny_vit_small_variant if small else tiny_vit_21m_variant
    enc = make(img_size=cfg["dataset"]["image_size"], use_checkpoint=True)
    model = TinyVideoMAE(enc, cfg)
    apply_rule(model)
    parity_mode(model)
    return model.to(DEV).train()


def _close(a, b, rtol, atol):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return bool(np.all(np.abs(a - b) <= atol + rtol * np.abs(b))), float(np.max(np.abs(a - b)))


def _run_steps(model, d, steps, bf16=False):
    from ssl_mae_amd.init_rule import synthetic_clip
    from ssl_mae_amd.optim import FusedAdamW, GradScaler
    from ssl_mae_amd.train_ssl_mae import train_step
    B, T, S = int(d["B"]), int(d["T"]), int(d["S"])
    opt = FusedAdamW(model.parameters(), lr=5e-4, weight_decay=0.05)
    scaler = GradScaler()
    torch.manual_seed(42)
    losses, preds, masks = [], [], []
    for i in range(steps):
        clip = torch.from_numpy(synthetic_clip(B, T, S, seed=int(d["clip_seed"]) + i)).to(DEV)
        loss, pred, idx = train_step(model, clip, opt, scaler, {"mask_ratio": float(d["ratio"]),
                                                                "norm_pix_loss": True}, bf16=bf16)
        torch.cuda.synchronize()
        losses.append(loss.item())
        preds.append(pred.detach().float().cpu())
        from ssl_mae_amd.mae_loader import tube_mask_with_index  # noqa: F401
    return losses, preds


GOLD = ["step_b2_t2_s32", "step_b2_t4_s64", "step_b1_t8_s224", "step_small_b2_t2_s32"]


@pytest.mark.parametrize("resident,lite", [((), ()), ((0, 1, 2), ()), ((1, 2), (0,))])
@pytest.mark.parametrize("case", GOLD)
def test_fp32_step_matches_reference_golden(golden_dir, case, resident, lite):
    """resident=(0, 1, 2): every stage kept in HBM (no checkpoint recompute); lite=(0,):
    stage 0 keeps only block inputs and recomputes a1/a2 in the backward.  Every policy
    must give the same loss, gradients, parameters and BN running stats (updated twice
    in stages 0-2, as the reference's checkpoint forward + recompute does)."""
    d = np.load(os.path.join(golden_dir, case + ".npz"))
    B, T, S = int(d["B"]), int(d["T"]), int(d["S"])
    small = "depths" in d.files and int(d["depths"][2]) == 12      # C3 "ViT-Small" 
    cfg = _cfg(B, T, S, float(d["ratio"]), int(d["decoder_depth"]) if "decoder_depth" in d.files else 4)
    model = _build(cfg, small)
    model.encoder.resident_stages = resident
    model.encoder.lite_stages = lite
    # mask parity first (bit-exact): same seed, same RNG stream as the reference's step
    from ssl_mae_amd.mae_loader import get_tube_mask
    torch.manual_seed(42)
    m = get_tube_mask(B, T, (S // 8) ** 2, float(d["ratio"]))
    assert np.array_equal(m.cpu().numpy(), d["mask"][0])
    losses, preds = _run_steps(model, d, 1)
    gl = float(d["avg_loss"])
    assert abs(losses[0] - gl) <= 1e-4 * max(1.0, abs(gl)), (losses[0], gl)
    pred = preds[0]
    if "pred" in d.files:
        ok, e = _close(pred.numpy(), d["pred"], 1e-3, 1e-3)
        assert ok, ("pred", e)
    ps = pred.double()
    ok, e = _close((ps * ps).sum().item(), d["pred_sumsq"], 1e-3, 0)
    assert ok, ("pred sumsq", e)
    # gradients (flat buffer views) against the reference's per-parameter checksums
    named = dict(model.named_parameters())
    n = 0
    for key in d.files:
        if not key.startswith("grad_sum/"):
            continue
        name = key[len("grad_sum/"):]
        g = named[name]._sm_grad.detach().double().cpu()
        scale = math.sqrt(float(d["grad_sumsq/" + name]))
        ok, e = _close((g * g).sum().item(), d["grad_sumsq/" + name], 2e-3, 1e-10)
        assert ok, (name, "sumsq", e)
        ok, e = _close(g.reshape(-1)[:8].numpy(), d["grad_head/" + name], 1e-3, 2e-4 * scale + 1e-7)
        assert ok, (name, "head", e)
        n += 1
    assert n == len([k for k in d.files if k.startswith("grad_sum/")]) and n >= 203
    # stage-4 params receive no gradient and are not updated (reference: grad None)
    for name, p in named.items():
        if name.startswith("encoder.stages.3."):
            assert p.grad is None
    # parameters after one AdamW step
    for name, p in named.items():
        gh = d["grad_head/" + name] if ("grad_head/" + name) in d.files else np.zeros(8)
        atol = np.where(np.abs(gh[: p.numel()]) < 1e-5, 2.1 * 5e-4, 2e-6)
        ok, e = _close(p.detach().reshape(-1)[:8].cpu().numpy(), d["param_head/" + name], 1e-5, atol)
        assert ok, (name, "param", e)
    # BN running stats: stem once, checkpointed stages 0-2 twice (reference checkpointing)
    bufs = dict(model.named_buffers())
    for key in d.files:
        if key.startswith("buf/"):
            name = key[4:]
            b = bufs[name].detach().cpu().numpy()
            ok, e = _close(b, d[key], 1e-3, 1e-4)
            assert ok, (name, e)


def test_fp32_two_steps_match_reference(golden_dir):
    d = np.load(os.path.join(golden_dir, "step2_b2_t2_s32.npz"))
    cfg = _cfg(int(d["B"]), int(d["T"]), int(d["S"]), float(d["ratio"]))
    model = _build(cfg)
    losses, _ = _run_steps(model, d, 2)
    assert abs(np.mean(losses) - float(d["avg_loss"])) < 1e-4
    for name, p in model.named_parameters():
        gh = d["grad_head/" + name] if ("grad_head/" + name) in d.files else np.zeros(8)
        atol = np.where(np.abs(gh[: p.numel()]) < 1e-5, 2 * 2.1 * 5e-4, 5e-5)
        ok, e = _close(p.detach().reshape(-1)[:8].cpu().numpy(), d["param_head/" + name], 1e-4, atol)
        assert ok, (name, e)


def test_bf16_step_close_to_oracle(golden_dir):
    """bf16 autocast path vs the fp32 reference: loss within 2 %, pred within 0.05 of
    its scale, per-parameter gradient cosine similarity > 0.98 for parameters
    carrying signal."""
    d = np.load(os.path.join(golden_dir, "step_b2_t4_s64.npz"))
    B, T, S = int(d["B"]), int(d["T"]), int(d["S"])
    cfg = _cfg(B, T, S, float(d["ratio"]))
    model = _build(cfg)
    losses, preds = _run_steps(model, d, 1, bf16=True)
    gl = float(d["avg_loss"])
    assert abs(losses[0] - gl) < 0.02 * abs(gl), (losses[0], gl)
    pr = preds[0].numpy()
    ref = d["pred"]
    assert np.max(np.abs(pr - ref)) < 0.05 * np.max(np.abs(ref)) + 0.05
    # gradient direction vs the oracle's full fp32 gradients
    from oracle import mae_oracle as O
    from ssl_mae_amd.init_rule import param_value, synthetic_clip
    P = O.make_params(cfg, param_value)
    clip = torch.from_numpy(synthetic_clip(B, T, S, seed=int(d["clip_seed"])))
    mask = torch.from_numpy(d["mask"][0])
    _, grads = O.train_step(P, None, None, clip, mask, cfg)
    named = dict(model.named_parameters())
    worst = 1.0
    for name, g in grads.items():
        if g is None:
            continue
        ours = named[name]._sm_grad.detach().double().cpu().reshape(-1)
        ref = g.double().reshape(-1)
        if ref.norm() < 1e-3 * max(1e-12, float(np.sqrt(d["grad_sumsq/" + name]))) or ref.norm() < 1e-6:
            continue
        cos = float(torch.dot(ours, ref) / (ours.norm() * ref.norm() + 1e-30))
        worst = min(worst, cos)
        assert cos > 0.98, (name, cos)


def test_forward_stage3_api_nchw(golden_dir):
    """TinyViT.forward_stage3 keeps the reference contract [N,3,H,W] -> [N,384,H/8,W/8]."""
    from ssl_mae_amd.init_rule import apply_rule, synthetic_clip
    from ssl_mae_amd.tiny_vit import tiny_vit_21m_variant
    d = np.load(os.path.join(golden_dir, "step_b2_t2_s32.npz"))
    B, T, S = int(d["B"]), int(d["T"]), int(d["S"])
    from ssl_mae_amd import parity_mode
    enc = parity_mode(tiny_vit_21m_variant(img_size=S))
    # the golden names are prefixed by 'encoder.'; apply the rule through a wrapper
    wrapper = torch.nn.Module()
    wrapper.encoder = enc
    apply_rule(wrapper)
    enc = enc.to(DEV).train()
    clip = torch.from_numpy(synthetic_clip(B, T, S, seed=int(d["clip_seed"]))).to(DEV)
    frames = clip.permute(0, 2, 1, 3, 4).reshape(B * T, 3, S, S)
    out = enc.forward_stage3(frames)
    assert out.shape == (B * T, 384, S // 8, S // 8)
    ok, e = _close(out.detach().cpu().numpy(), d["act_stage2"], 1e-3, 1e-3)
    assert ok, e


def test_patchify_unpatchify_roundtrip_and_golden(golden_dir):
    from ssl_mae_amd.train_ssl_mae import patchify, unpatchify
    d = np.load(os.path.join(golden_dir, "patchify.npz"))
    shape = tuple(int(s) for s in d["patchify_in_shape"])
    x = torch.arange(int(np.prod(shape)), dtype=torch.float32).reshape(shape).to(DEV)
    out = patchify(x, 8)
    assert np.array_equal(out.cpu().numpy(), d["patchify_out"])
    back = unpatchify(out, *shape[1:], p=8)
    assert torch.equal(back, x)


def test_training_regularisers_active_and_replayable():
    """Dropout (decoder) and DropPath (encoder) are on in train mode: the loss differs
    from the parity-mode loss, is identical for identical seeds, and a second step
    draws new masks."""
    from ssl_mae_amd.init_rule import apply_rule, synthetic_clip
    from ssl_mae_amd.mae_vit_adapter import TinyVideoMAE
    from ssl_mae_amd.tiny_vit import tiny_vit_21m_variant
    from ssl_mae_amd import parity_mode
    cfg = _cfg(2, 2, 32, 0.75)
    clip = torch.from_numpy(synthetic_clip(2, 2, 32, seed=3)).to(DEV)
    mask = torch.zeros(2, 2, 16, dtype=torch.bool, device=DEV)
    mask[:, :, :12] = True

    def loss_of(parity, seed):
        torch.manual_seed(seed)
        m = TinyVideoMAE(tiny_vit_21m_variant(img_size=32), cfg)
        apply_rule(m)
        if parity:
            parity_mode(m)
        m = m.to(DEV).train()
        from ssl_mae_amd.functions import mae_loss
        with torch.autocast("cuda", dtype=torch.bfloat16):
            pred = m(clip, mask)
        l1 = mae_loss(pred, clip, mask).item()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            pred = m(clip, mask)
        return l1, mae_loss(pred, clip, mask).item()

    a1, a2 = loss_of(False, 0)
    b1, b2 = loss_of(False, 0)
    p1, p2 = loss_of(True, 0)
    assert a1 == b1 and a2 == b2          # replayable from the seed
    assert a1 != a2                        # new masks each forward
    assert p1 == p2                        # parity mode is deterministic
    assert a1 != p1
