"""Per-op roofline ledger of one bench training step (B=256 by default).

Every public function of ssl_mae_amd.kernels is wrapped with HIP events on the
current stream (outermost call only).  Per (op, shapes) group the ledger prints
calls, measured ms, the op's tensor bytes (every distinct tensor argument and
output, counted once: the algorithmic HBM floor), GEMM/attention FLOP, the ideal
time max(bytes / 8 TB/s, flop / 2.5 PF) and the gap to it.  Sorted by gap.

    python scripts/ledger.py [--batch 256] [--top 60]
"""
import argparse
import functools
import inspect
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ssl-vit-video-analytics_amd")]

import torch  # noqa: E402

HBM = 8.0e12
MFMA = 2.5e15


def _flop(name, ba):
    a = ba.arguments
    if name == "gemm":
        return 2.0 * a["M"] * a["N"] * a["K"]
    if name == "linear":
        return 2.0 * a["x"].shape[0] * a["x"].shape[1] * a["w"].shape[0]
    if name == "linear_dx":
        return 2.0 * a["dy"].shape[0] * a["dy"].shape[1] * a["w"].shape[1]
    if name == "linear_dw":
        return 2.0 * a["dy"].shape[0] * a["dy"].shape[1] * a["x"].shape[1]
    if name == "attn_fwd":
        return 4.0 * a["N"] * a["H"] * a["L"] ** 2 * a["D"]
    if name == "attn_bwd":   # algorithmic (2x forward), not the 14x the split kernels execute
        return 8.0 * a["N"] * a["H"] * a["L"] ** 2 * a["D"]
    return 0.0


def _tensors(x, out):
    if isinstance(x, torch.Tensor):
        out.append(x)
    elif isinstance(x, (tuple, list)):
        for y in x:
            _tensors(y, out)
    return out


def install(K, records):
    depth = [0]
    for name, fn in list(vars(K).items()):
        if name.startswith("_") or not inspect.isfunction(fn) or fn.__module__ != K.__name__:
            continue
        sig = inspect.signature(fn)

        def make(name=name, fn=fn, sig=sig):
            @functools.wraps(fn)
            def w(*a, **k):
                if depth[0] or not records.active:
                    return fn(*a, **k)
                depth[0] += 1
                try:
                    s = torch.cuda.Event(enable_timing=True)
                    e = torch.cuda.Event(enable_timing=True)
                    s.record()
                    out = fn(*a, **k)
                    e.record()
                finally:
                    depth[0] -= 1
                ba = sig.bind(*a, **k)
                ts = _tensors(list(ba.arguments.values()), [])
                ts = _tensors(out, ts)
                seen, nbytes = set(), 0
                for t in ts:
                    key = (t.data_ptr(), t.numel())
                    if key not in seen:
                        seen.add(key)
                        nbytes += t.numel() * t.element_size()
                shp = []
                for n, v in ba.arguments.items():
                    if isinstance(v, torch.Tensor):
                        shp.append(f"{n}{list(v.shape)}{str(v.dtype)[6:][:4]}")
                    elif isinstance(v, bool) and v:
                        shp.append(n)
                    elif isinstance(v, int) and not isinstance(v, bool) and n != "seed" and abs(v) < 1 << 31:
                        shp.append(f"{n}={v}")
                    elif isinstance(v, float) and n in ("drop_p",) and v > 0:
                        shp.append(f"{n}={v}")
                records.rows.append((name, " ".join(shp), s, e, nbytes, _flop(name, ba)))
                return out
            return w
        setattr(K, name, make())


class Records:
    def __init__(self):
        self.rows = []
        self.active = False


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--top", type=int, default=60)
    ap.add_argument("--arena", default="on", choices=["on", "off"],
                    help="the device-memory arena, as bench.py's MAE step runs (its memory policy follows)")
    args = ap.parse_args()
    if args.arena == "on":
        from ssl_mae_amd import arena
        arena.install()
    from ssl_mae_amd import kernels as K
    from ssl_mae_amd.build import build
    build()
    rec = Records()
    install(K, rec)
    from ssl_mae_amd.optim import FusedAdamW, GradScaler
    from ssl_mae_amd.train_ssl_mae import build_model, train_step
    dev = torch.device("cuda", 0)
    B, T, S = args.batch, 8, 224
    cfg = {"dataset": {"clip_len": T, "image_size": S, "stride": 4, "train_split": "-"},
           "model": {"decoder_embed_dim": 384, "decoder_depth": 4, "decoder_num_heads": 6},
           "ssl": {"mask_ratio": 0.75, "norm_pix_loss": True},
           "training": {"batch_size": B, "lr": 5e-4, "log_interval": 20}}
    torch.manual_seed(1234)
    model = build_model(cfg, dev).train()
    opt = FusedAdamW(model.parameters(), lr=5e-4, weight_decay=0.05)
    clip = torch.randn(B, 3, T, S, S, device=dev)
    train_step(model, clip, opt, GradScaler(), cfg["ssl"], bf16=True)
    torch.cuda.synchronize()
    rec.active = True
    s0 = torch.cuda.Event(enable_timing=True)
    e0 = torch.cuda.Event(enable_timing=True)
    s0.record()
    train_step(model, clip, opt, GradScaler(), cfg["ssl"], bf16=True)
    e0.record()
    torch.cuda.synchronize()
    rec.active = False
    step_ms = s0.elapsed_time(e0)
    groups = {}
    for name, shp, s, e, nb, fl in rec.rows:
        g = groups.setdefault((name, shp), [0, 0.0, 0, 0.0])
        g[0] += 1
        g[1] += s.elapsed_time(e)
        g[2] += nb
        g[3] += fl
    tot = sum(g[1] for g in groups.values())
    ideal_tot = sum(max(g[2] / HBM, g[3] / MFMA) * 1e3 for g in groups.values())
    print(f"step {step_ms:.1f} ms; ops {tot:.1f} ms; ideal (roofline floor of the same ops) {ideal_tot:.1f} ms")
    rows = []
    for (name, shp), (n, ms, nb, fl) in groups.items():
        ideal = max(nb / HBM, fl / MFMA) * 1e3
        rows.append((ms - ideal, name, shp, n, ms, nb, fl, ideal))
    rows.sort(reverse=True)
    print(f"{'gap ms':>8} {'ms':>8} {'ideal':>7} {'n':>3} {'GB/s':>6} {'TF/s':>6}  op")
    for gap, name, shp, n, ms, nb, fl, ideal in rows[:args.top]:
        print(f"{gap:8.1f} {ms:8.1f} {ideal:7.1f} {n:3d} {nb / ms / 1e6:6.0f} {fl / ms / 1e9:6.0f}  {name} {shp}")


if __name__ == "__main__":
    main()
