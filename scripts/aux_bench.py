"""Time the kernels of the rows next to the hot path:

* FedAvg aggregation (sm_fedavg_weighted_sum) at BASELINE config C5: 4 clients x
  the full MAE state (TinyViT-21M variant + 4x384 decoder, fp32).  Algorithmic
  bytes per launch = (K + 1) x n x 4 (K client reads + one write).
* clip normalisation (sm_frames_normalize) at the bench batch: 256 clips x 8 frames
  x 224^2.  Algorithmic bytes = 3 (uint8 RGB read) + 12 (3 fp32 written) per pixel.

Prints one JSON line per kernel; run under rocprofv3 --kernel-trace --stats to
cross-check the average launch durations."""
import json
import os
import sys

import torch

sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                             "ssl-vit-video-analytics_amd")]
from ssl_mae_amd import federated as F  # noqa: E402
from ssl_mae_amd import kernels as K  # noqa: E402


def _time(fn, iters):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def frames(B=256, T=8, S=224, iters=30):
    f = torch.randint(0, 256, (B, T, S, S, 3), dtype=torch.uint8, device="cuda")
    out = torch.empty((B, 3, T, S, S), dtype=torch.float32, device="cuda")
    ms = _time(lambda: K.frames_normalize(f, (0.485, 0.456, 0.406), (0.229, 0.224, 0.225), True, None, out), iters)
    gb = B * T * S * S * 15 / 1e9
    print(json.dumps({"kernel": "frames_norm4_kernel", "clips": B, "frames": T, "size": S,
                      "avg_launch_ms": round(ms, 4), "algorithmic_gb_per_launch": round(gb, 4),
                      "achieved_gbs": round(gb / ms * 1e3, 1), "peak_gbs": 8000.0,
                      "frac": round(gb / ms * 1e3 / 8000.0, 3)}))


def main(k=4, iters=50):
    from ssl_mae_amd.mae_vit_adapter import TinyVideoMAE
    from ssl_mae_amd.tiny_vit import tiny_vit_21m_variant
    cfg = {"dataset": {"clip_len": 8, "image_size": 224},
           "model": {"decoder_embed_dim": 384, "decoder_depth": 4, "decoder_num_heads": 6}}
    m = TinyVideoMAE(tiny_vit_21m_variant(img_size=224), cfg)
    n = sum(v.numel() for v in m.state_dict().values() if v.is_floating_point())
    bufs = [torch.randn(n, device="cuda") for _ in range(k)]
    w = F._norm_weights([1.0 + i for i in range(k)], float(sum(1.0 + i for i in range(k))))
    out = torch.empty_like(bufs[0])
    for _ in range(5):
        K.fedavg_weighted_sum(bufs, w, out)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        K.fedavg_weighted_sum(bufs, w, out)
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / iters
    gb = (k + 1) * n * 4 / 1e9
    print(json.dumps({"kernel": "fedavg_sum4_kernel", "clients": k, "elements": n, "avg_launch_ms": round(ms, 4),
                      "algorithmic_gb_per_launch": round(gb, 4), "achieved_gbs": round(gb / ms * 1e3, 1),
                      "peak_gbs": 8000.0, "frac": round(gb / ms * 1e3 / 8000.0, 3)}))


if __name__ == "__main__":
    main()
    frames()
