"""BASELINE config 4: fine-tune with the frozen HIP encoder + linear head (16-frame
clips, 112x112), against the golden recorded by running the reference's TinyViT
(tests/golden/make_golden_finetune.py): the linear-probe training step under
model.train() (per-frame batch statistics, running stats updated once per frame
call, AdamW on the head) and the evaluation forward under model.eval() (running
statistics, all four stages through TinyViT.forward).  fp32 mode: 1e-3 (north
star tolerance); bf16 autocast: 3e-2 of the logit scale."""
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


def _close(a, b, rtol, atol):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return bool(np.all(np.abs(a - b) <= atol + rtol * np.abs(b))), float(np.max(np.abs(a - b)))


def _model(nc):
    from ssl_mae_amd.finetune import VideoClassifier
    from ssl_mae_amd.init_rule import apply_rule
    m = VideoClassifier(nc, img_size=112)
    apply_rule(m)
    for mod in m.modules():
        if hasattr(mod, "drop_prob"):
            mod.drop_prob = 0.0
    return m.to(DEV)


def _golden(golden_dir):
    return np.load(os.path.join(golden_dir, "finetune_b2_t16_s112.npz"))


def test_linear_probe_step_and_eval_match_reference(golden_dir):
    from ssl_mae_amd.finetune import set_requires_grad
    from ssl_mae_amd.init_rule import synthetic_clip
    d = _golden(golden_dir)
    B, T, S, NC = int(d["B"]), int(d["T"]), int(d["S"]), int(d["num_classes"])
    model = _model(NC)
    set_requires_grad(model.backbone, False)
    opt = torch.optim.AdamW([p for p in model.parameters() if p.requires_grad], lr=1e-3, weight_decay=0.01)
    clip = torch.from_numpy(synthetic_clip(B, T, S, seed=4321)).to(DEV)
    label = torch.tensor([3, 77], device=DEV)
    model.train()
    opt.zero_grad(set_to_none=True)
    logits = model(clip)
    loss = torch.nn.CrossEntropyLoss()(logits, label)
    loss.backward()
    ok, e = _close(logits.detach().cpu().numpy(), d["train_logits"], 1e-3, 1e-3)
    assert ok, ("train logits", e)
    assert abs(loss.item() - float(d["train_loss"])) < 1e-4 * max(1.0, float(d["train_loss"]))
    ok, e = _close(model.classifier.weight.grad.cpu().numpy(), d["head_grad_w"], 1e-3, 1e-5)
    assert ok, ("head grad w", e)
    ok, e = _close(model.classifier.bias.grad.cpu().numpy(), d["head_grad_b"], 1e-3, 1e-6)
    assert ok, ("head grad b", e)
    assert all(p.grad is None for p in model.backbone.parameters())       # frozen: no backbone grads
    opt.step()
    # Adam normalises g / (|g| + eps): near-zero gradient entries may move by up to 2 lr
    gw = d["head_grad_w"]
    ok, e = _close(model.classifier.weight.detach().cpu().numpy(), d["head_w_after"], 1e-5,
                   np.where(np.abs(gw) < 1e-5, 2.1e-3, 2e-6))
    assert ok, ("head w", e)
    ok, e = _close(model.classifier.bias.detach().cpu().numpy(), d["head_b_after"], 1e-5, 2e-6)
    assert ok, ("head b", e)
    bufs = dict(model.backbone.named_buffers())
    n = 0
    for key in d.files:
        if key.startswith("buf/"):
            name = key[4:]
            got = bufs[name].detach().cpu().numpy()
            if name.endswith("num_batches_tracked"):
                assert int(got) == T, name
            else:
                ok, e = _close(got, d[key], 1e-3, 1e-4)
                assert ok, (name, e)
            n += 1
    assert n == 3 * (2 + 3 * 5)          # 2 stem BNs + 3 per MBConv (5 MBConvs in 4 stages)
    # evaluation: running statistics, all B*T frames in one batch
    clip2 = torch.from_numpy(synthetic_clip(B, T, S, seed=8765)).to(DEV)
    model.eval()
    with torch.no_grad():
        frames = clip2.permute(0, 2, 1, 3, 4).reshape(B * T, 3, S, S)
        feat, emb = model.backbone(frames)
        logits2 = model(clip2)
    assert tuple(feat.shape) == tuple(int(v) for v in d["eval_feat_shape"])
    f = feat.double()
    assert abs(f.sum().item() - float(d["eval_feat_sum"])) <= 1e-3 * abs(float(d["eval_feat_sumsq"])) ** 0.5 * 10
    assert abs((f * f).sum().item() / float(d["eval_feat_sumsq"]) - 1) < 1e-3
    ok, e = _close(emb.cpu().numpy(), d["eval_emb"], 1e-3, 1e-3)
    assert ok, ("eval emb", e)
    ok, e = _close(logits2.cpu().numpy(), d["eval_logits"], 1e-3, 1e-3)
    assert ok, ("eval logits", e)
    # bf16 autocast (the benchmarked precision) on the same eval clip
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        lb = model(clip2)
    ref = d["eval_logits"]
    assert np.max(np.abs(lb.float().cpu().numpy() - ref)) < 3e-2 * np.max(np.abs(ref)) + 3e-2


def test_full_finetune_backward_runs_through_encoder():
    """ft_ssl mode (backbone trainable, train-mode BN): gradients reach every
    backbone parameter through the fused backward (stage 4 included) and are finite."""
    from ssl_mae_amd.init_rule import synthetic_clip
    model = _model(11).train()
    clip = torch.from_numpy(synthetic_clip(2, 4, 112, seed=3)).to(DEV)
    opt = torch.optim.AdamW(model.parameters(), lr=1e-4)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        logits = model(clip)
    loss = torch.nn.CrossEntropyLoss()(logits.float(), torch.tensor([1, 7], device=DEV))
    loss.backward()
    for n, p in model.named_parameters():
        assert p.grad is not None and torch.isfinite(p.grad).all(), n
    assert model.backbone.stages[3][1].attn.qkv.weight.grad.abs().sum() > 0
    opt.step()


def test_train_mode_droppath_masks_differ_across_frame_calls():
    """Each per-frame backbone call of a train-mode forward draws its own DropPath
    masks (the reference's per-call torch RNG draws).  The same frame repeated at
    every t gives identical per-frame embeddings with DropPath off (control) and
    different ones with it on."""
    from ssl_mae_amd.finetune import frame_modes
    from ssl_mae_amd.functions import Mode
    from ssl_mae_amd.init_rule import synthetic_clip
    ms = frame_modes(Mode(True, 1234), 4)
    assert len({m.seed_base for m in ms}) == 4
    frame = torch.from_numpy(synthetic_clip(4, 1, 112, seed=5)).to(DEV)
    clip = frame.expand(4, 3, 4, 112, 112).contiguous()
    for p_drop in (0.0, 0.5):
        model = _model(5).train()
        for mod in model.modules():
            if hasattr(mod, "drop_prob"):
                mod.drop_prob = p_drop
        captured = []
        orig = model.backbone.embed

        def spy(x, mode, frames=None, _orig=orig):
            out = _orig(x, mode)
            captured.append(out[0].detach().float().clone())
            return out
        model.backbone.embed = spy
        with torch.no_grad():
            model(clip)
        assert len(captured) == 4
        diffs = [float((captured[t] - captured[0]).abs().max()) for t in range(1, 4)]
        if p_drop == 0.0:
            assert max(diffs) == 0.0, diffs
        else:
            assert min(diffs) > 0.0, diffs


def test_ft_ssl_backbone_gradients_match_reference(golden_dir):
    """ft_ssl mode (train_finetune.py:198-210: backbone trainable), fp32, DropPath 0:
    one training step's gradient of EVERY backbone parameter -- the sum of the T
    per-frame fused backward groups written into the flat gradient buffer -- against
    the reference's TinyViT run (tests/golden/make_golden_finetune.py ftssl).  Per
    parameter: L2 norm within 1e-3 relative, sum and first 8 values within 1e-3 of
    the reference value plus 1e-3 of the parameter's gradient RMS (cancellation)."""
    from ssl_mae_amd.init_rule import synthetic_clip
    d = np.load(os.path.join(golden_dir, "finetune_ftssl_b2_t2_s112.npz"))
    B, T, S, NC = int(d["B"]), int(d["T"]), int(d["S"]), int(d["num_classes"])
    model = _model(NC).train()
    clip = torch.from_numpy(synthetic_clip(B, T, S, seed=2468)).to(DEV)
    logits = model(clip)
    loss = torch.nn.CrossEntropyLoss()(logits, torch.tensor([1, 7], device=DEV))
    loss.backward()
    ok, e = _close(logits.detach().cpu().numpy(), d["logits"], 1e-3, 1e-3)
    assert ok, ("logits", e)
    assert abs(loss.item() - float(d["loss"])) < 1e-3 * abs(float(d["loss"]))
    params = dict(model.named_parameters())
    names = [str(n) for n in d["names"]]
    assert sum(n.startswith("backbone.") for n in names) > 150
    bad = []
    top = max(float(d["gl2/" + n]) for n in names)
    for n in names:
        g = params[n].grad
        assert g is not None, n
        g = g.detach().double().reshape(-1).cpu()
        l2, ref_l2 = float(g.norm()), float(d["gl2/" + n])
        if ref_l2 < 1e-5 * top:
            # analytically ~zero (a bias feeding a train-mode BatchNorm): rounding noise
            # on both sides; only its size is checked
            if l2 > 1e-4 * top:
                bad.append((n, "noise", l2, top))
            continue
        rms = ref_l2 / max(1, g.numel()) ** 0.5
        if abs(l2 - ref_l2) > 1e-3 * ref_l2 + 1e-9:
            bad.append((n, "l2", l2, ref_l2))
        if abs(float(g.sum()) - float(d["gsum/" + n])) > 1e-3 * abs(float(d["gsum/" + n])) + 1e-3 * rms * g.numel() ** 0.5:
            bad.append((n, "sum", float(g.sum()), float(d["gsum/" + n])))
        h = g[:8].numpy()
        ref_h = d["ghead/" + n]
        if np.any(np.abs(h - ref_h) > 1e-3 * np.abs(ref_h) + 1e-3 * rms):
            bad.append((n, "head", float(np.max(np.abs(h - ref_h))), rms))
    assert not bad, bad[:10]
