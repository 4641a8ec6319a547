"""Generate tests/golden/bf16_anchor_b1_t8_s224.npz by RUNNING the reference twice: its own
forward + backward at the C2 clip (B=1, T=8, 224^2, the step_b1_t8_s224 clip, init rule and
tube mask) in fp32 and under bf16 autocast, recording how far the reference's OWN bf16 run
lands from its fp32 run: per-stage activation errors (stem, stages 0-2, pred; relative L2
and relative max), the loss, and per-parameter gradient cosines / norm ratios.
tests/test_bf16_pin_gpu.py gates the timed bf16 kernels at <= 1.5x these numbers.

The reference trains under torch.amp.autocast('cuda', dtype=torch.bfloat16)
(src/train_ssl_mae.py:79-84).  This container has no GPU, so the reference runs under
torch.autocast('cpu', dtype=torch.bfloat16): the same lower-precision set for the
matmul-class ops (conv2d, linear, matmul / bmm inside attention), fp32 for the rest.
Parity mode as make_golden.py (dropout / DropPath p = 0, BN in train mode).  Runs ONLY in
the build container (the reference never travels); output is data only.

    python tests/golden/make_golden_bf16.py
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as MG  # noqa: E402
from ssl_mae_amd.init_rule import apply_rule, synthetic_clip  # noqa: E402


def run(ref, bf16, B=1, T=8, S=224, ratio=0.75, clip_seed=1234):
    tiny_vit, adapter, mae_loader, ref_utils, tr = ref
    torch.set_num_threads(8)
    cfg = MG.make_config(T, S, ratio, batch=B)
    model = adapter.TinyVideoMAE(tiny_vit.tiny_vit_21m_variant(img_size=S, use_checkpoint=True), cfg)
    apply_rule(model)
    MG._parity_mode(model)
    model.train()
    clip = torch.from_numpy(synthetic_clip(B, T, S, seed=clip_seed))
    acts = {}

    def grab(key):
        def h(mod, inp, out):
            if key not in acts:
                acts[key] = out.detach().float().clone()
        return h
    hooks = [model.encoder.patch_embed.register_forward_hook(grab("act_stem"))]
    for i in range(3):
        hooks.append(model.encoder.stages[i].register_forward_hook(grab(f"act_stage{i}")))
    hooks.append(model.register_forward_hook(grab("pred")))
    ref_utils.set_seed(42)
    L = (S // 8) * (S // 8)
    mask = mae_loader.get_tube_mask(B, T, L, ratio)
    # train_ssl_mae.py:72-84, with the autocast region on the CPU
    target = tr.patchify(clip, p=8)
    mean = target.mean(dim=-1, keepdim=True)
    var = target.var(dim=-1, keepdim=True)
    target = (target - mean) / (var + 1.e-6) ** .5
    with torch.autocast("cpu", dtype=torch.bfloat16, enabled=bf16):
        pred = model(clip, mask)
        loss_map = ((pred - target) ** 2).mean(dim=-1)
        mf = mask.flatten(1, 2)
        loss = (loss_map * mf).sum() / (mf.sum() + 1e-6)
    loss.backward()
    for h in hooks:
        h.remove()
    grads = {n: p.grad.detach().double().clone() for n, p in model.named_parameters() if p.grad is not None}
    return acts, float(loss), grads


def main():
    ref = MG._import_reference()
    a32, l32, g32 = run(ref, False)
    a16, l16, g16 = run(ref, True)
    rec = {"B": 1, "T": 8, "S": 224, "clip_seed": 1234, "loss_fp32": l32, "loss_bf16": l16}
    for k in a32:
        x, y = a16[k].double().reshape(-1), a32[k].double().reshape(-1)
        rec["rel_l2/" + k] = float((x - y).norm() / (y.norm() + 1e-30))
        rec["rel_max/" + k] = float((x - y).abs().max() / (y.abs().max() + 1e-30))
        print(f"{k:12s} rel L2 {rec['rel_l2/' + k]:.3e}  rel max {rec['rel_max/' + k]:.3e}")
    gmax = max(float(g.abs().max()) for g in g32.values())
    names, cos, ratio = [], [], []
    for n, g in g32.items():
        h = g16[n]
        if float(g.norm()) < 1e-5 * gmax:   # analytically zero (bias feeding a train-mode BN): noise
            continue
        names.append(n)
        cos.append(float(torch.dot(h.reshape(-1), g.reshape(-1)) / (h.norm() * g.norm() + 1e-30)))
        ratio.append(float(h.norm() / (g.norm() + 1e-30)))
    rec["grad_names"] = np.array(names)
    rec["grad_cos"] = np.array(cos)
    rec["grad_norm_ratio"] = np.array(ratio)
    allg32 = torch.cat([g32[n].reshape(-1) for n in names])
    allg16 = torch.cat([g16[n].reshape(-1) for n in names])
    rec["grad_cos_all"] = float(torch.dot(allg16, allg32) / (allg16.norm() * allg32.norm()))
    print(f"loss fp32 {l32:.6f} bf16 {l16:.6f} (rel {abs(l16 - l32) / abs(l32):.2e}); grad cos min "
          f"{min(cos):.4f} (5th pct {np.percentile(cos, 5):.4f}), all {rec['grad_cos_all']:.6f}; "
          f"norm ratio {min(ratio):.3f}..{max(ratio):.3f}")
    out = os.path.join(HERE, "bf16_anchor_b1_t8_s224.npz")
    np.savez_compressed(out, **rec)
    print("wrote", out)


if __name__ == "__main__":
    main()
