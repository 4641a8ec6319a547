"""Benchmark: clips/s of the MAE pretraining step (BASELINE.json config 2:
ViT-Tiny (TinyViT-21M variant) MAE, bf16, batch 256 per GPU, 8x3x224x224
synthetic clips, mask ratio 0.75) on N GPUs of one node.

One step = tube mask + forward (bf16 autocast) + fused masked-recon loss +
backward + data-parallel gradient all-reduce (N > 1) + AdamW, exactly the body of
train_one_epoch (train_ssl_mae.py:66-91) with inputs already resident in HBM.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...

Rank 0 prints one JSON line (see the driver contract in DESIGN.md).
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "ssl-vit-video-analytics_amd")
for _p in (ROOT, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "clips/sec (8x3x224x224) MAE ViT-Tiny pretrain, 1/2/4/8 GPU + recon-loss parity"
FWD_GFLOP_PER_CLIP = 739.0            # SURVEY.md §8(d), T=8, 224^2 (MATH-SDPA FlopCounter)
TRAIN_TFLOP_PER_CLIP = 3 * FWD_GFLOP_PER_CLIP / 1000.0
MFMA_BF16_PEAK_TFLOPS = 2500.0        # MI355X dense bf16 (MI355X_MICROARCH.md)
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=256, help="clips per GPU")
    ap.add_argument("--frames", type=int, default=8)
    ap.add_argument("--size", type=int, default=224)
    ap.add_argument("--mask-ratio", type=float, default=0.75)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--attn-bwd-shape", default="",
                    help="A/B only: MFMA shape of the bf16 attention backward as 'D64,D32' (16 or 32 each; "
                         "default: the library's); reported in config when given")
    ap.add_argument("--no-calibration", action="store_true",
                    help="skip the box calibration (bare MFMA loops + a 4.9 GB copy) before the timed steps")
    ap.add_argument("--resident", default="",
                    help="encoder stages kept resident in HBM (no checkpoint recompute): "
                         "comma list, or 'none'; default: the model's auto policy")
    ap.add_argument("--lite", default="",
                    help="encoder stages kept lite-resident (MBConv a1/a2 recomputed in the backward instead of "
                         "the whole stage): comma list or 'none'; default: the model's auto policy")
    ap.add_argument("--arena", default="auto", choices=["auto", "on", "off"],
                    help="device-memory arena (ssl_mae_amd/arena.py) instead of the caching allocator: "
                         "auto = on for the MAE step (its stage-0 resident policy needs the arena's "
                         "coalescing heap), off for the fine-tune step")
    ap.add_argument("--probe", default="dec_attn_bwd",
                    help="kernel group timed with events for the roofline line: dec_attn_bwd (the top-time "
                         "kernels of the step: decoder attention dK/dV + dQ) or dec_attn_fwd")
    ap.add_argument("--model", default="tiny", choices=["tiny", "small"],
                    help="tiny: tiny_vit_21m_variant + 4-layer decoder (BASELINE C2); small: the build-defined "
                         "ViT-Small of BASELINE C3 (depths 2,2,12,2 + 8-layer decoder, SURVEY.md H8)")
    ap.add_argument("--workload", default="mae", choices=["mae", "finetune"],
                    help="mae: MAE pretraining step (C2/C3); finetune: frozen-encoder linear-probe step "
                         "(BASELINE C4: 16-frame 112x112 clips, batch 64)")
    return ap.parse_args()


def _cpu_point(T, S, ratio, B, th):
    """One point of cpu_baseline (run in a child process): the oracle's fp32 fwd+bwd+AdamW step
    of the C1 step shape on B clips with torch on `th` threads, after a small warm-up step."""
    from oracle import mae_oracle as O
    from ssl_mae_amd.init_rule import param_value, synthetic_clip
    torch.set_num_threads(th)
    cfg = {"dataset": {"clip_len": T, "image_size": S},
           "model": {"decoder_embed_dim": 384, "decoder_depth": 4, "decoder_num_heads": 6},
           "ssl": {"mask_ratio": ratio, "norm_pix_loss": True}, "train_dropout": True}
    wcfg = dict(cfg, dataset={"clip_len": 2, "image_size": 64})
    torch.manual_seed(42)
    wP = O.make_params(wcfg, param_value)
    O.train_step(wP, O.init_buffers(wP), O.AdamWState(lr=5e-4), torch.from_numpy(synthetic_clip(1, 2, 64, seed=6)),
                 O.get_tube_mask(1, 2, 64, ratio), wcfg)
    del wP
    P = O.make_params(cfg, param_value)
    bufs = O.init_buffers(P)
    opt = O.AdamWState(lr=5e-4)
    clip = torch.from_numpy(synthetic_clip(B, T, S, seed=7))
    mask = O.get_tube_mask(B, T, (S // 8) ** 2, ratio)
    t0 = time.perf_counter()
    O.train_step(P, bufs, opt, clip, mask, cfg)
    dt = time.perf_counter() - t0
    return {"clips": B, "threads": th, "s_per_step": round(dt, 2), "clips_per_s": round(B / dt, 5)}


def cpu_baseline(T, S, ratio, sweep=((1, 16), (1, 32), (1, 64)), budget_s=45.0, point_timeout_s=75.0):
    """The CPU oracle (fp32 restatement of the reference path, oracle/mae_oracle.py) timed on
    the GPU box's host cores: one fwd+bwd+AdamW step of the reference's C1 step shape
    (train_ssl_mae.py:66-91, T=8, 224^2) per (clips, threads) point of `sweep`, with dropout /
    DropPath on as the reference ships them (attention probabilities materialised per head, as
    nn.MultiheadAttention's math path), after an untimed small warm-up step.  A bounded sample:
    one clip per point (the reference's 4-clip C1 batch takes minutes), each point in a child
    process with a time limit (the box is a share of a 256-CPU host whose other tenants can make
    a wide thread pool stall: 256 threads did), further points only while the sweep has used less
    than `budget_s`.  The headline value is the fastest point; the reference's own B = 4 step is
    cpu_baseline_reference."""
    import subprocess
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = os.cpu_count()
    points = []
    t_start = time.perf_counter()
    for B, th in sweep:
        th = min(th, affinity)
        if points and (time.perf_counter() - t_start > budget_s or any(p.get("threads") == th for p in points)):
            break
        print(f"[bench] cpu baseline: {B} clip(s) on {th} threads", file=sys.stderr, flush=True)
        code = (f"import json, sys; sys.path[:0] = {[ROOT, PKG]!r}; import bench; "
                f"print(json.dumps(bench._cpu_point({T}, {S}, {ratio}, {B}, {th})))")
        try:
            r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                               timeout=point_timeout_s, env=dict(os.environ, OMP_NUM_THREADS=str(th)))
            points.append(json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else
                          {"clips": B, "threads": th, "error": r.stderr[-200:]})
        except subprocess.TimeoutExpired:
            points.append({"clips": B, "threads": th, "timeout_s": point_timeout_s})
    ok = [p for p in points if "clips_per_s" in p]
    if not ok:
        return {"value": None, "unit": "clips/s", "kind": "port", "sweep": points}
    head = max(ok, key=lambda p: p["clips_per_s"])
    return {"value": head["clips_per_s"], "unit": "clips/s", "cores": head["threads"], "threads": head["threads"],
            "nproc": os.cpu_count(), "affinity_cpus": affinity, "kind": "port", "sweep": points,
            "sample": f"BASELINE config 1 step shape: one fp32 fwd+bwd+AdamW step of oracle/mae_oracle.py on "
                      f"{head['clips']} clip ({T}x3x{S}x{S}) with dropout / DropPath on (as the reference), after a "
                      f"small warm-up step; fastest of the thread counts in 'sweep' ({head['threads']} threads, "
                      f"{head['s_per_step']} s).  The box is a 1-GPU share of a host whose affinity set shows "
                      f"{affinity} CPUs (nproc {os.cpu_count()}); the harness sizes a GPU's CPU share at 16 "
                      f"(OMP_NUM_THREADS=16 on the box)"}


def calibration(dev, copy_gb=4.9):
    """Box calibration before the timed steps (~2 s): bare bf16 MFMA loops on random register
    data in both shapes (csrc/calib.hip; TFLOP/s and the in-kernel clock, MI355X_MICROARCH.md
    'DVFS give-back' items 5-7: devices differ by up to 12 % on the same MFMA loop) and a
    device-to-device copy of `copy_gb` GB (read + write bytes / time), so a line from a slow box
    can be told from slow code."""
    from ssl_mae_amd import kernels as K
    out = {}
    for shape, name in ((32, "32x32x16"), (16, "16x16x32")):
        tf, mhz, ms = K.calibrate_mfma(shape, iters=1_500_000)
        out[f"mfma_{name}_tflops"] = round(tf, 1)
        out[f"mfma_{name}_clock_mhz"] = round(mhz) if mhz else None
        out[f"mfma_{name}_ms"] = round(ms, 1)
    n = int(copy_gb * 1e9) // 4
    src = torch.empty(n, dtype=torch.float32, device=dev).uniform_()
    dst = torch.empty_like(src)
    dst.copy_(src)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(3):
        dst.copy_(src)
    e.record()
    e.synchronize()
    ms = s.elapsed_time(e) / 3
    out["copy_gbs"] = round(2 * n * 4 / (ms * 1e-3) / 1e9, 1)
    out["copy_gb"] = copy_gb
    del src, dst
    return out


PROBE_KERNELS = {"dec_attn_fwd": "attn_fwd_bf16<64, true>",
                 "dec_attn_bwd": "attn_bwd_dq_bf16<64, true, 4>+attn_bwd_dkdv_bf16<64, true, 4>",
                 "dec_attn_bwd16": "attn_bwd_dq16_bf16<64, true, 4>+attn_bwd_dkdv16_bf16<64, true, 4>"}
def reference_cpu():
    """The reference's own train_one_epoch timed on the build container's CPU cores at
    BASELINE config 1 by scripts/ref_cpu_baseline.py (the reference cannot travel to
    the GPU box); the newest committed profiles/*_ref_cpu_baseline.json."""
    import glob
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_ref_cpu_baseline.json")), reverse=True):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        out = {k: d[k] for k in ("value", "unit", "cores", "kind", "sample") if k in d}
        out["source"] = os.path.relpath(f, ROOT)
        return out
    return None


def probe_kernel_key(probe):
    """PROBE_KERNELS key of the kernels the probe times: the decoder backward's kernel pair
    depends on the MFMA shape selected for head dim 64 (sm_attn_tuning)."""
    if probe == "dec_attn_bwd":
        from ssl_mae_amd import kernels as K
        return "dec_attn_bwd16" if K.attn_tuning(64) == 16 else "dec_attn_bwd"
    return probe


def pmc_traffic(probe, B, T, S):
    """HBM bytes per launch of the probe kernel(s), measured with PMC counters by
    scripts/pmc_traffic.sh (FETCH_SIZE / WRITE_SIZE passes over this bench at the
    default workload) and committed as profiles/*_traffic.json; None if absent."""
    import glob
    if (B, T, S) != (256, 8, 224):
        return None
    L = T * (S // 8) ** 2
    qkv, o, lse = B * L * 3 * 384 * 2, B * L * 384 * 2, B * 6 * L * 4
    algo = {"dec_attn_fwd": qkv + o + lse,                       # qkv read + O write + lse
            "dec_attn_bwd": qkv + 2 * o + lse + qkv}             # qkv, O, dO, lse read + dqkv write
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_traffic.json")), reverse=True):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if d.get("kernel") == PROBE_KERNELS.get(probe_kernel_key(probe)):
            return {"traffic": round(d["traffic_bytes"] / 1e9, 3), "traffic_unit": "GB/launch",
                    "algorithmic_gb_per_launch": round(algo[probe] / 1e9, 3),
                    "traffic_source": os.path.relpath(f, ROOT)}
    return None


class Probe:
    """HIP-event timing of one kernel group on the stream it is launched on."""

    def __init__(self, name):
        self.name = name
        self.pairs = []
        self.active = False

    def wrap(self, mod, fn_name, select):
        orig = getattr(mod, fn_name)
        probe = self

        def wrapped(*a, **k):
            if probe.active and select(*a, **k):
                s = torch.cuda.Event(enable_timing=True)
                e = torch.cuda.Event(enable_timing=True)
                s.record()
                out = orig(*a, **k)
                e.record()
                probe.pairs.append((s, e))
                return out
            return orig(*a, **k)
        setattr(mod, fn_name, wrapped)

    def avg_ms(self):
        if not self.pairs:
            return None
        return sum(s.elapsed_time(e) for s, e in self.pairs) / len(self.pairs)


def resident_used(model, frames, S):
    from ssl_mae_amd.tiny_vit import auto_resident_stages
    enc = model.encoder
    r = enc.resident_stages
    return auto_resident_stages(frames, S, True, torch.device("cuda"), key=(tuple(enc.depths), enc._sm_dec_depth)) \
        if r == "auto" else r


def lite_used(model, frames, S):
    from ssl_mae_amd.tiny_vit import auto_lite_stages
    enc = model.encoder
    if enc.lite_stages != "auto":
        return list(enc.lite_stages)
    return list(auto_lite_stages(frames, S, True, torch.device("cuda"), resident_used(model, frames, S),
                                 key=(tuple(enc.depths), enc._sm_dec_depth)))


def main():
    args = parse()
    if args.arena == "on" or (args.arena == "auto" and args.workload == "mae"):
        from ssl_mae_amd import arena as smarena
        # before the first CUDA allocation of the process; ranks of a multi-GPU run
        # leave RCCL's channel buffers 8 GiB outside the heap
        smarena.install(reserve_mib=8192 if int(os.environ.get("WORLD_SIZE", "1")) > 1 else None)
    from ssl_mae_amd import dist as smdist
    from ssl_mae_amd import kernels as K
    from ssl_mae_amd.build import build
    rank, world = smdist.init_from_env()
    if world == 1 and args.gpus > 1 and rank == 0:
        print(f"[bench] --gpus {args.gpus} without torchrun: running one process", file=sys.stderr)
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if rank == 0:
        build()
    if world > 1:
        dist.barrier()

    from ssl_mae_amd.init_rule import IMAGENET_MEAN, IMAGENET_STD
    from ssl_mae_amd.optim import FusedAdamW, GradScaler
    from ssl_mae_amd.train_ssl_mae import build_model, train_step

    if args.workload == "finetune":
        return bench_finetune(args, rank, world, dev)
    B, T, S, r = args.batch, args.frames, args.size, args.mask_ratio
    small = args.model == "small"
    cfg = {"dataset": {"clip_len": T, "image_size": S, "stride": 4, "train_split": "-"},
           "model": {"decoder_embed_dim": 384, "decoder_depth": 8 if small else 4, "decoder_num_heads": 6,
                     "encoder": "tiny_vit_small_variant" if small else "tiny_vit_21m_variant"},
           "ssl": {"mask_ratio": r, "norm_pix_loss": True},
           "training": {"batch_size": B, "lr": 5e-4, "log_interval": 20}}
    torch.manual_seed(1234)
    model = build_model(cfg, dev).train()
    if args.resident:
        model.encoder.resident_stages = () if args.resident == "none" else \
            tuple(int(v) for v in args.resident.split(","))
    if args.lite:
        model.encoder.lite_stages = () if args.lite == "none" else tuple(int(v) for v in args.lite.split(","))
    torch.manual_seed(4321 + rank)               # per-rank mask stream
    opt = FusedAdamW(model.parameters(), lr=5e-4, weight_decay=0.05)
    scaler = GradScaler()
    # synthetic clips resident in HBM: (U[0,1) - mean_c) / std_c, per rank
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    mean = torch.tensor(IMAGENET_MEAN, device=dev).view(1, 3, 1, 1, 1)
    std = torch.tensor(IMAGENET_STD, device=dev).view(1, 3, 1, 1, 1)
    clips = [((torch.rand(B, 3, T, S, S, generator=g, device=dev) - mean) / std) for _ in range(2)]

    probe = Probe(args.probe)
    stem_probe = Probe("patch_embed_fwd")
    from ssl_mae_amd import tiny_vit as TV
    stem_probe.wrap(TV.PatchEmbed, "run", lambda *a, **k: True)
    Ld = T * (S // 8) ** 2
    if args.probe == "dec_attn_fwd":
        probe.wrap(K, "attn_fwd", lambda qkv, N, L, H, D, *a, **k: D == 64 and L == Ld)
        flop_per_launch = 4.0 * B * 6 * Ld * Ld * 64        # S = QK^T and O = PV
        exec_flop_per_launch = flop_per_launch
    elif args.probe == "dec_attn_bwd":
        probe.wrap(K, "attn_bwd", lambda qkv, o, do, lse, N, L, H, D, *a, **k: D == 64 and L == Ld)
        # training work = 3x forward, so the backward's algorithmic work
        # is 2x the forward's 4*B*H*L^2*D (dV, dP, dQ, dK; the recompute of S is not
        # counted).  The split dK/dV + dQ kernels execute 14*B*H*L^2*D (S and dP in both).
        flop_per_launch = 8.0 * B * 6 * Ld * Ld * 64
        exec_flop_per_launch = 14.0 * B * 6 * Ld * Ld * 64
    else:
        flop_per_launch = exec_flop_per_launch = None

    ssl_cfg = cfg["ssl"]
    # rank-0 weights/buffers broadcast; bucketed RCCL all-reduce launched from the
    # backward on a side stream (N > 1)
    smdist.setup_data_parallel(model, opt, world)

    def step(i):
        loss, _, _ = train_step(model, clips[i % 2], opt, scaler, ssl_cfg, bf16=True)
        return loss

    if args.attn_bwd_shape:
        for D, v in zip((64, 32), args.attn_bwd_shape.split(",")):
            K.attn_tuning(D, int(v))
    if args.resident or args.lite:   # an explicit policy must fit before the first step (RuntimeError)
        enc = model.encoder
        TV.check_memory_policy(B * T, S, True, dev, resident_used(model, B * T, S), lite_used(model, B * T, S),
                               key=(tuple(enc.depths), enc._sm_dec_depth))
    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    print(f"[bench] {args.warmup} warm-up steps done", file=sys.stderr, flush=True)
    calib = None
    if not args.no_calibration:
        try:
            calib = calibration(dev)
        except Exception as e:   # the calibration must not cost the bench line
            calib = {"error": repr(e)[:200]}
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    probe.active = True
    stem_probe.active = True
    t0 = time.perf_counter()
    loss_vals, step_end = [], []
    for i in range(args.steps):
        # the reference syncs on the loss every step (total_loss += loss.item(),
        # train_ssl_mae.py:91): so does the timed loop
        loss_vals.append(float(step(i).item()))
        step_end.append(time.perf_counter())
        if rank == 0 and (i + 1) % 10 == 0:
            print(f"[bench] {i + 1}/{args.steps} timed steps", file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    probe.active = False
    stem_probe.active = False
    if world > 1:
        dist.barrier()
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    from ssl_mae_amd import arena as smarena
    peak_mem = smarena.max_memory_allocated(dev) / 2 ** 30
    if smarena.active() and os.environ.get("SM_BENCH_MEMSTATS"):
        print("[bench] arena: " + " ".join(f"{k}={v}" for k, v in smarena.stats(dev).items()), file=sys.stderr)
    if os.environ.get("SM_BENCH_SNAPSHOT") and not smarena.active():   # caching-allocator segments (diagnostics)
        segs = torch.cuda.memory_snapshot()
        summary = [{"size": sg["total_size"], "allocated": sg["allocated_size"], "stream": sg.get("stream"),
                    "blocks": [(b["size"], b["state"]) for b in sg["blocks"]][:64]} for sg in segs]
        with open(os.environ["SM_BENCH_SNAPSHOT"], "w") as fh:
            json.dump(summary, fh)
    if os.environ.get("SM_BENCH_MEMSTATS") and not smarena.active():   # allocator behaviour (A/B diagnostics)
        ms_ = torch.cuda.memory_stats(dev)
        print("[bench] allocator: " + " ".join(f"{k}={ms_.get(k)}" for k in (
            "num_alloc_retries", "num_device_alloc", "num_device_free", "num_sync_all_streams",
            "reserved_bytes.all.peak", "allocated_bytes.all.peak")), file=sys.stderr)

    if rank == 0:
        clips_total = B * world * args.steps
        value = clips_total / elapsed
        ms = elapsed / args.steps * 1e3
        roof = None
        avg = probe.avg_ms()
        if avg and flop_per_launch:
            achieved = flop_per_launch / (avg * 1e-3) / 1e12
            roof = {"kernel": args.probe, "kernels": PROBE_KERNELS.get(probe_kernel_key(args.probe)),
                    "bound": "mfma", "achieved": round(achieved, 1),
                    "peak": MFMA_BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
                    "frac": round(achieved / MFMA_BF16_PEAK_TFLOPS, 4), "traffic": None,
                    "avg_launch_ms": round(avg, 3), "launches": len(probe.pairs),
                    "algorithmic_flop_per_launch": flop_per_launch,
                    "executed_flop_per_launch": exec_flop_per_launch,
                    "executed_frac": round(exec_flop_per_launch / (avg * 1e-3) / 1e12 / MFMA_BF16_PEAK_TFLOPS, 4)}
            tr = pmc_traffic(args.probe, B, T, S)
            if tr:
                roof.update(tr)
        savg = stem_probe.avg_ms()
        if roof is not None and savg:
            # north star: achieved HBM GB/s of the patch-embed stem (forward launch:
            # conv1 + BN + GELU + conv2 + BN), algorithmic bytes SURVEY.md §8(d):
            # fp32 clip in (3*T*H*W*4) + bf16 [frames,112,112,96] out = 24.1 MB/clip
            sbytes = B * (3 * T * S * S * 4 + 96 * T * (S // 2) * (S // 2) * 2)
            roof["patch_embed"] = {"bound": "hbm", "achieved": round(sbytes / (savg * 1e-3) / 1e9, 1),
                                   "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                   "frac": round(sbytes / (savg * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                   "algorithmic_gb_per_launch": round(sbytes / 1e9, 3),
                                   "avg_launch_ms": round(savg, 3), "launches": len(stem_probe.pairs)}
        step_tflops = value / world * TRAIN_TFLOP_PER_CLIP if not small else None
        cpu = None
        if not args.no_cpu_baseline and world == 1 and not small:
            try:
                cpu = cpu_baseline(T, S, r)
            except Exception as e:  # the baseline must not kill the bench line
                cpu = {"value": None, "error": repr(e)[:200]}
        step_ms = [round((b_ - a_) * 1e3, 1) for a_, b_ in zip([t0] + step_end[:-1], step_end)]
        line = {
            "metric": METRIC, "value": round(value, 3), "unit": "clips/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 2),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
            "data": "synthetic (U[0,1) ImageNet-normalised clips in HBM; random-init weights)",
            "config": {"workload": ("BASELINE config 3: build-defined ViT-Small MAE (TinyViT depths 2,2,12,2, "
                                    "stem+stages 1-3) + 8x384 decoder" if small else
                                    "BASELINE config 2: TinyViT-21M-variant MAE (stem+stages 1-3) + 4x384 decoder")
                                   + ", T=8, 224x224, mask 0.75, bf16 autocast",
                       "model": ("tiny_vit_small_variant" if small else "tiny_vit_21m_variant") + " + TinyVideoMAE",
                       "global_batch": B * world,
                       "per_gpu_batch": B, "frames": T, "image_size": S, "mask_ratio": r,
                       "parallelism": f"dp{world}",
                       "resident_stages": list(resident_used(model, B * T, S)),
                       "lite_stages": lite_used(model, B * T, S),
                       **({"gemm_tuning": K.gemm_tuning_nondefault()} if K.gemm_tuning_nondefault() else {}),
                       **({"attn_bwd_shape": args.attn_bwd_shape} if args.attn_bwd_shape else {})},
            "calibration": calib,
            "step_ms_first5": step_ms[:5], "step_ms_last5": step_ms[-5:],
            "roofline": roof,
            "model_tflops_per_gpu": round(step_tflops, 1) if step_tflops else None,
            "model_mfu": round(step_tflops / MFMA_BF16_PEAK_TFLOPS, 4) if step_tflops else None,
            "peak_mem_gib": round(peak_mem, 1),
            "allocator": ({"kind": "arena", "capacity_gib": round(smarena.stats(dev)["capacity"] / 2 ** 30, 1),
                           "hipmalloc_requests": smarena.stats(dev)["hipmalloc_requests"]}
                          if smarena.active() else {"kind": "caching"}),
            "loss_first_last": [round(loss_vals[0], 5), round(loss_vals[-1], 5)],
            "loss_item_per_step": True,
            "cpu_baseline": cpu,
            "cpu_baseline_reference": reference_cpu() if not small else None,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def bench_finetune(args, rank, world, dev):
    """BASELINE config 4: the linear-probe training step of train_finetune.py
    (:84-124, mode linear_probe :294-296): VideoClassifier with the frozen HIP TinyViT
    encoder (all four stages, train-mode BatchNorm per frame call as the reference),
    temporal mean, Linear head, CE loss, AdamW on the head; bf16 autocast.  Batch 64
    clips (configs/finetune.yaml) of 16 frames at 112x112.  Also times the evaluation
    forward (model.eval(), no_grad)."""
    from ssl_mae_amd.finetune import VideoClassifier, set_requires_grad
    from ssl_mae_amd.init_rule import IMAGENET_MEAN, IMAGENET_STD
    B, T, S, NC = 64, 16, 112, 101
    torch.manual_seed(1234)
    model = VideoClassifier(NC, img_size=S).to(dev)
    set_requires_grad(model.backbone, False)
    opt = torch.optim.AdamW([p for p in model.parameters() if p.requires_grad], lr=1e-4, weight_decay=0.01)
    g = torch.Generator(device=dev).manual_seed(99 + rank)
    mean = torch.tensor(IMAGENET_MEAN, device=dev).view(1, 3, 1, 1, 1)
    std = torch.tensor(IMAGENET_STD, device=dev).view(1, 3, 1, 1, 1)
    clip = (torch.rand(B, 3, T, S, S, generator=g, device=dev) - mean) / std
    label = torch.randint(0, NC, (B,), generator=g, device=dev)
    ce = torch.nn.CrossEntropyLoss()

    def train_step():
        model.train()
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            logits = model(clip)
        loss = ce(logits.float(), label)
        loss.backward()
        opt.step()
        return loss

    def timed(fn, steps, warmup):
        for _ in range(warmup):
            fn()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            out = fn()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([el], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = t.item()
        return el, out

    el, loss = timed(train_step, args.steps, args.warmup)

    def eval_step():
        model.eval()
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
            return model(clip)
    el_eval, _ = timed(eval_step, args.steps, 1)
    if rank == 0:
        value = B * world * args.steps / el
        line = {"metric": "clips/sec (16x3x112x112) frozen-encoder fine-tune step (linear probe)",
                "value": round(value, 3), "unit": "clips/s", "n_gpus": world, "steps": args.steps,
                "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 2), "higher_is_better": True,
                "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
                "data": "synthetic (U[0,1) ImageNet-normalised clips in HBM; random-init weights)",
                "config": {"workload": "BASELINE config 4: VideoClassifier(frozen TinyViT-21M-variant encoder, all 4 "
                                       "stages, train-mode BN per frame call) + Linear(576, 101), CE + AdamW on "
                                       "the head, T=16, 112x112, bf16 autocast",
                           "global_batch": B * world, "per_gpu_batch": B, "frames": T, "image_size": S,
                           "parallelism": f"dp{world}"},
                "eval_clips_per_s": round(B * world * args.steps / el_eval, 2),
                "loss_last": round(float(loss.item()), 5),
                "peak_mem_gib": round(torch.cuda.max_memory_allocated(dev) / 2 ** 30, 1)}
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
