"""Measure how far the timed bf16 path sits from fp32 references (to set the tolerances of
tests/test_bf16_pin_gpu.py from data):

  1. B=1, T=8, 224^2: bf16 HIP step's stage outputs (stem y, stages 0-2) and pred against
     the fp32 CPU oracle's on the same clip / mask (relative L2 and max errors);
  2. B=N, T=8, 224^2 (default 32): bf16 HIP step vs the fp32-mode HIP step (exact-fp32
     kernels, pinned to 1e-3 of the reference golden) on the same clips, mask and
     dropout / DropPath masks: loss, per-parameter gradient cosine and norm ratio.

python scripts/bf16_pin_probe.py [--batch 32] [--skip-oracle]
"""
import argparse
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ssl-vit-video-analytics_amd")]

import torch  # noqa: E402

DEV = "cuda"


def cfg_of(B, T, S):
    return {"dataset": {"clip_len": T, "image_size": S, "stride": 4, "train_split": "-"},
            "model": {"decoder_embed_dim": 384, "decoder_depth": 4, "decoder_num_heads": 6},
            "ssl": {"mask_ratio": 0.75, "norm_pix_loss": True},
            "training": {"batch_size": B, "lr": 5e-4, "log_interval": 20}}


def model_of(cfg, parity):
    from ssl_mae_amd import parity_mode
    from ssl_mae_amd.init_rule import apply_rule
    from ssl_mae_amd.mae_vit_adapter import TinyVideoMAE
    from ssl_mae_amd.tiny_vit import tiny_vit_21m_variant
    torch.manual_seed(42)
    m = TinyVideoMAE(tiny_vit_21m_variant(img_size=cfg["dataset"]["image_size"]), cfg)
    apply_rule(m)
    if parity:
        parity_mode(m)
    return m.to(DEV).train()


def capture(stages_out):
    """Record PatchEmbed / stage outputs of the first forward (channels-last, BN applied)."""
    from ssl_mae_amd import kernels as K
    from ssl_mae_amd import tiny_vit as TV
    pe_run, st_run = TV.PatchEmbed.run, TV._Stage.run

    def pe(self, clip, mode):
        t, xbn = pe_run(self, clip, mode)
        if "act_stem" not in stages_out:
            y = t if xbn is None else K.bn_apply(t.reshape(-1, t.shape[-1]), *xbn[:4], gelu=False).view(t.shape)
            stages_out["act_stem"] = y.detach().float().clone()
        return t, xbn

    def st(self, x, mode, resident=False, x_bn=None):
        out = st_run(self, x, mode, resident, x_bn)
        key = f"act_stage{self._probe_stage}"
        if key not in stages_out:
            stages_out[key] = out.detach().float().clone()
        return out
    TV.PatchEmbed.run, TV._Stage.run = pe, st
    return lambda: (setattr(TV.PatchEmbed, "run", pe_run), setattr(TV._Stage, "run", st_run))


def errs(a, b):
    a, b = a.double().cpu().reshape(-1), b.double().cpu().reshape(-1)
    return (a - b).norm().item() / (b.norm().item() + 1e-30), (a - b).abs().max().item() / (b.abs().max().item() + 1e-30)


def step(model, clip, bf16, seed=42):
    from ssl_mae_amd.optim import FusedAdamW, GradScaler
    from ssl_mae_amd.train_ssl_mae import train_step
    opt = FusedAdamW(model.parameters(), lr=5e-4, weight_decay=0.05)
    torch.manual_seed(seed)
    torch.cuda.synchronize()
    t0 = time.time()
    loss, pred, idx = train_step(model, clip, opt, GradScaler(), model._probe_cfg["ssl"], bf16=bf16)
    torch.cuda.synchronize()
    grads = {n: p._sm_grad.detach().double().cpu().clone() for n, p in model.named_parameters()
             if getattr(p, "_sm_grad", None) is not None and ".stages.3." not in n}
    return loss.item(), pred.detach(), grads, time.time() - t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--skip-oracle", action="store_true")
    ap.add_argument("--parity", action="store_true", help="dropout / DropPath off in part 2")
    args = ap.parse_args()
    from ssl_mae_amd import _lib
    from ssl_mae_amd.init_rule import synthetic_clip
    _lib.load()
    if not args.skip_oracle:
        from oracle import mae_oracle as O
        from ssl_mae_amd.init_rule import param_value
        cfg = cfg_of(1, 8, 224)
        model = model_of(cfg, True)
        model._probe_cfg = cfg
        for i, s in enumerate(model.encoder.stages):
            s._probe_stage = i
        clip = torch.from_numpy(synthetic_clip(1, 8, 224, seed=1234)).to(DEV)
        ours = {}
        undo = capture(ours)
        torch.manual_seed(42)
        from ssl_mae_amd.mae_loader import tube_mask_with_index
        mask, _ = tube_mask_with_index(1, 8, 784, 0.75, device=DEV)
        torch.manual_seed(42)
        loss, pred, grads, dt = step(model, clip, True)
        undo()
        ours["pred"] = pred.float()
        P = O.make_params(cfg, param_value)
        acts = {}
        t0 = time.time()
        O.train_step(P, None, None, clip.cpu(), mask.cpu(), cfg, acts=acts)
        print(f"oracle step {time.time() - t0:.1f} s", flush=True)
        for k in ("act_stem", "act_stage0", "act_stage1", "act_stage2", "pred"):
            ref = acts[k]
            got = ours[k]
            if k != "pred":
                got = got.permute(0, 3, 1, 2)
            l2, mx = errs(got, ref)
            print(f"B=1 {k:11s} rel L2 {l2:.3e}  rel max {mx:.3e}", flush=True)
    B = args.batch
    cfg = cfg_of(B, 8, 224)
    clip = torch.from_numpy(synthetic_clip(B, 8, 224, seed=77)).to(DEV)
    res = {}
    for bf16 in (False, True):
        model = model_of(cfg, args.parity)
        model._probe_cfg = cfg
        res[bf16] = step(model, clip, bf16)
        print(f"B={B} {'bf16' if bf16 else 'fp32'} loss {res[bf16][0]:.6f}  step {res[bf16][3]:.1f} s", flush=True)
        del model
        torch.cuda.empty_cache()
    lf, lb = res[False][0], res[True][0]
    print(f"B={B} loss rel diff {abs(lb - lf) / abs(lf):.3e}", flush=True)
    gf, gb = res[False][2], res[True][2]
    worst = []
    for n, g in gf.items():
        h = gb[n]
        nf = g.norm().item()
        if nf < 1e-8:
            continue
        cos = float(torch.dot(g.reshape(-1), h.reshape(-1)) / (nf * h.norm().item() + 1e-30))
        worst.append((cos, abs(h.norm().item() / nf - 1), n))
    worst.sort()
    for c, r, n in worst[:12]:
        print(f"  cos {c:.5f}  |norm ratio - 1| {r:.4f}  {n}", flush=True)
    print(f"B={B} params {len(worst)}  min cos {worst[0][0]:.5f}  max norm dev {max(w[1] for w in worst):.4f}",
          flush=True)
    # loss of the first clips inside the B-clip bf16 run vs a separate fp32 run on them
    print("pred shapes", res[True][1].shape, flush=True)


if __name__ == "__main__":
    main()
