"""Time the REFERENCE's own training step on this container's CPU cores at BASELINE
config 1 (ViT-Tiny MAE = tiny_vit_21m_variant + 4x384 decoder, B=4, T=8, 224x224,
mask 0.75, fp32 -- autocast('cuda') / GradScaler('cuda') disable themselves on a
CPU-only box -- dropout and DropPath ON as shipped).

The reference is imported exactly as tests/golden/make_golden.py does it (timm.layers
stand-in, torchvision/tensorboard placeholders, mae_loader by file path) and its
`train_one_epoch` (src/train_ssl_mae.py:52-123) runs over a list of synthetic clips
(its loader is the data pipeline, which SURVEY.md §8(d) excludes).  The model is
built as main() builds it (set_seed(42), :131,143-144).  Runs ONLY in the build
container (the reference never travels to the GPU box); bench.py reports the
committed result as `cpu_baseline_reference`.

    python scripts/ref_cpu_baseline.py [--steps 3] [--threads 8] [--out profiles/r03_ref_cpu_baseline.json]
"""
import argparse
import json
import os
import platform
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests", "golden"), os.path.join(ROOT, "ssl-vit-video-analytics_amd")]


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


class TimedClips:
    """The step inputs as train_one_epoch's `loader`, stamping the start of each step."""

    def __init__(self, clips):
        self.clips, self.stamps = clips, []

    def __len__(self):
        return len(self.clips)

    def __iter__(self):
        for c in self.clips:
            self.stamps.append(time.perf_counter())
            yield c
        self.stamps.append(time.perf_counter())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r03_ref_cpu_baseline.json"))
    args = ap.parse_args()
    import make_golden as MG
    from ssl_mae_amd.init_rule import synthetic_clip
    tiny_vit, adapter, _, ref_utils, tr = MG._import_reference()
    torch.set_num_threads(args.threads)
    B, T, S, r = 4, 8, 224, 0.75
    cfg = MG.make_config(T, S, r, batch=B)
    ref_utils.set_seed(42)
    model = adapter.TinyVideoMAE(tiny_vit.tiny_vit_21m_variant(img_size=S, use_checkpoint=True), cfg)
    optimizer = torch.optim.AdamW(model.parameters(), lr=5e-4, weight_decay=0.05)
    scaler = torch.amp.GradScaler("cuda")
    clips = TimedClips([torch.from_numpy(synthetic_clip(B, T, S, seed=1234 + i)) for i in range(args.steps)])
    avg_loss, _ = tr.train_one_epoch(model, clips, optimizer, scaler, 1, torch.device("cpu"), cfg,
                                     MG._Writer(), MG._Logger())
    st = clips.stamps
    per_step = [b - a for a, b in zip(st[:-1], st[1:])]
    timed = per_step[1:] if len(per_step) > 1 else per_step      # first step = warm-up
    sec = sum(timed) / len(timed)
    rec = {"value": round(B / sec, 5), "unit": "clips/s", "cores": args.threads, "kind": "reference",
           "sample": f"the reference's train_one_epoch (src/train_ssl_mae.py:52-123) itself at BASELINE config 1: "
                     f"B={B}, T={T}, {S}x{S}, mask {r}, fp32, dropout/DropPath on, {len(timed)} timed step(s) after "
                     f"{len(per_step) - len(timed)} warm-up on {args.threads} threads of the build container "
                     f"({cpu_model()}); {sec:.1f} s per step",
           "seconds_per_step": [round(v, 2) for v in per_step], "avg_loss": avg_loss,
           "torch": torch.__version__, "script": "scripts/ref_cpu_baseline.py"}
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
