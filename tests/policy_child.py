"""Child process of tests/test_policy_gpu.py: the benchmarked memory policy, exactly as
bench.py runs it (device-memory arena installed before the first CUDA allocation, B = 256
clips of 8 x 224^2, bf16 autocast, dropout / DropPath on, FusedAdamW + GradScaler), against
the same step under the caching-allocator-era policy (stages 1-2 resident, stage 0 lite) on
the same clips, mask and dropout seeds.

python tests/policy_child.py -> one JSON line: per policy the loss, the reference loss formula
(train_ssl_mae.py:26-31,72-84) evaluated in fp32 torch on the step's own pred and mask, the BN
counters, whether every gradient is finite, and sha256 digests of the flat parameters after
AdamW, the flat gradients and every BN running buffer; plus the arena's counters."""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [HERE, os.path.join(HERE, "ssl-vit-video-analytics_amd")]

B, T, S = 256, 8, 224


def _digest(t):
    return hashlib.sha256(t.detach().contiguous().cpu().view(-1).view(dtype=__import__("torch").uint8).numpy()
                          .tobytes()).hexdigest()


def run_policy(resident, lite, clip, cfg, dev):
    import torch
    from ssl_mae_amd import arena
    from ssl_mae_amd.optim import FusedAdamW, GradScaler
    from ssl_mae_amd.train_ssl_mae import build_model, train_step
    torch.manual_seed(1234)
    model = build_model(cfg, dev).train()
    model.encoder.resident_stages = resident
    model.encoder.lite_stages = lite
    opt = FusedAdamW(model.parameters(), lr=5e-4, weight_decay=0.05)
    torch.manual_seed(4321)                       # bench.py's mask stream (rank 0)
    loss, pred, idx = train_step(model, clip, opt, GradScaler(), cfg["ssl"], bf16=True)
    lv = float(loss.item())
    L = T * (S // 8) ** 2
    x = clip.reshape(B, 3, T, S // 8, 8, S // 8, 8).permute(0, 2, 3, 5, 4, 6, 1)
    tgt = x.reshape(B, L, 192)
    tgt = (tgt - tgt.mean(-1, keepdim=True)) / torch.sqrt(tgt.var(-1, keepdim=True) + 1e-6)
    m = torch.zeros(B * L, device=dev)
    m[idx.long()] = 1.0
    per_tok = ((pred.float() - tgt) ** 2).mean(-1).reshape(-1)
    ref = float((per_tok.double() * m.double()).sum() / (m.double().sum() + 1e-6))
    del x, tgt, m, per_tok, pred
    flat = model._sm_flat
    counters = {n: int(b) for n, b in model.named_buffers() if n.endswith("num_batches_tracked")}
    bufs = hashlib.sha256()
    for n, b in sorted(model.named_buffers()):
        if not n.endswith("num_batches_tracked"):
            bufs.update(_digest(b).encode())
    out = {"resident": list(resident), "lite": list(lite), "loss": lv, "ref_loss": ref,
           "mask_rows": int(idx.numel()), "grad_finite": bool(torch.isfinite(flat.grad[:flat.used_end]).all()),
           "params": _digest(flat.data[:flat.used_end]), "grads": _digest(flat.grad[:flat.used_end]),
           "buffers": bufs.hexdigest(), "counters": counters, "peak_gib": arena.stats(dev)["peak"] / 2 ** 30}
    del model, opt, flat, loss, idx
    arena.library().sm_arena_reset_peak(dev.index)
    return out


def main():
    import torch
    from ssl_mae_amd import arena
    arena.install()
    from ssl_mae_amd.init_rule import IMAGENET_MEAN, IMAGENET_STD
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    cfg = {"dataset": {"clip_len": T, "image_size": S, "stride": 4, "train_split": "-"},
           "model": {"decoder_embed_dim": 384, "decoder_depth": 4, "decoder_num_heads": 6,
                     "encoder": "tiny_vit_21m_variant"},
           "ssl": {"mask_ratio": 0.75, "norm_pix_loss": True},
           "training": {"batch_size": B, "lr": 5e-4, "log_interval": 20}}
    g = torch.Generator(device=dev).manual_seed(1234)   # bench.py's clips (rank 0)
    mean = torch.tensor(IMAGENET_MEAN, device=dev).view(1, 3, 1, 1, 1)
    std = torch.tensor(IMAGENET_STD, device=dev).view(1, 3, 1, 1, 1)
    clip = (torch.rand(B, 3, T, S, S, generator=g, device=dev) - mean) / std
    from ssl_mae_amd.tiny_vit import auto_resident_stages, auto_lite_stages
    auto_r = auto_resident_stages(B * T, S, True, dev)
    auto_l = auto_lite_stages(B * T, S, True, dev, auto_r)
    res = [run_policy(tuple(auto_r), tuple(auto_l), clip, cfg, dev),
           run_policy((1, 2), (0,), clip, cfg, dev)]
    print(json.dumps({"auto": [list(auto_r), list(auto_l)], "runs": res, "arena": arena.stats(dev)}), flush=True)


if __name__ == "__main__":
    main()
