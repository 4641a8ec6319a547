"""MAE pretraining driver (reference: src/train_ssl_mae.py), MI355X-native.

`patchify(imgs, p)` and `train_one_epoch(model, loader, optimizer, scaler, epoch,
device, config, writer, logger)` keep the reference's signatures and per-step
semantics (train_ssl_mae.py:52-123): tube mask -> forward under bf16 autocast ->
masked normalised-pixel MSE -> zero_grad / backward / step -> `loss.item()` every
step, and every `log_interval` steps the masked-prediction std and throughput
(log_interval * batch_size / elapsed).  `main()` honours `--config` (the
reference hard-codes the path, :130) and runs the loop the reference's :168
TypeError prevents.  The loader is the MI355X clip pipeline of mae_loader
(uint8 frames, one H2D copy, sm_frames_normalize on the GPU); a loader that yields
ready fp32 clips (the reference's transform path) is accepted as well.  Every 10
epochs the reference's encoder-only file is written, plus a full training-state
file (`checkpoint.py`) that `--resume` continues from.

Data parallel (north star; the reference is single-device, :132): launched under
torchrun, `main()` runs one process per GPU (RCCL over xGMI, `dist.init_from_env`),
shards the dataset with a DistributedSampler (`set_epoch` per epoch), starts every
replica from rank 0's weights and all-reduces the gradients in buckets on a side
stream during the backward (`dist.setup_data_parallel`).  BatchNorm keeps
per-replica batch statistics.  The logged loss is the mean over ranks, the logged
throughput the global samples/s; logs and checkpoints are written by rank 0 only.
With one process it is exactly the single-device loop.
"""
import argparse
import logging
import os
import time
from datetime import timedelta
from pathlib import Path

import torch
import torch.distributed as dist

from . import dist as smdist
from . import ops as K    # every kernel launch through the torch.ops.ssl_mae dispatcher
from .functions import mae_loss, masked_pred_std
from .checkpoint import gather_rng_states, load_training_state, save_training_state
from .mae_loader import ClipNormalizer, LazyVideoMAEDataset, collate_frames, tube_mask_with_index
from .mae_vit_adapter import TinyVideoMAE
from .optim import FusedAdamW, GradScaler
from .tiny_vit import ENCODERS
from .utils import load_config, save_checkpoint, set_seed


def format_time(seconds):
    return str(timedelta(seconds=int(seconds)))


def patchify(imgs, p=8):
    """[B,C,T,H,W] -> [B, T*(H/p)*(W/p), p*p*C]; token (t,h,w), feature (pi,qi,c)."""
    return K.patchify(imgs, p)


def unpatchify(tokens, C, T, H, W, p=8):
    """Exact inverse of patchify (the reference's visualize_mae.py:30 einsum drops q)."""
    return K.unpatchify(tokens, C, T, H, W, p)


def setup_logger(save_dir):
    log_dir = Path("logs") / Path(save_dir).name
    log_dir.mkdir(parents=True, exist_ok=True)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s - %(levelname)s - %(message)s",
                        handlers=[logging.FileHandler(log_dir / "train.log"), logging.StreamHandler()])
    return logging.getLogger(__name__), log_dir


class NullWriter:
    def add_scalar(self, *a, **k):
        pass


def train_step(model, clip, optimizer, scaler, ssl_cfg, bf16=True):
    """One iteration of train_one_epoch's body; returns (loss tensor, pred, mask index)."""
    B, C, T, H, W = clip.shape
    L = (H // 8) * (W // 8)
    mask, idx = tube_mask_with_index(B, T, L, ssl_cfg["mask_ratio"], device=clip.device)
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=bf16):
        pred = model(clip, mask)
    loss = mae_loss(pred, clip, mask, ssl_cfg.get("norm_pix_loss", True))
    optimizer.zero_grad()
    scaler.scale(loss).backward()
    scaler.step(optimizer)
    scaler.update()
    return loss, pred, idx


def _to_clip(batch, device, normalizer):
    """A loader batch -> fp32 clip [B,3,T,H,W] on the device: (uint8 frames, valid)
    from the transform=None dataset goes through sm_frames_normalize; a tensor is a
    ready clip (reference transform path)."""
    if isinstance(batch, (tuple, list)):
        frames, valid = batch
        return normalizer(frames, valid)
    return batch.to(device, non_blocking=True)


def _world():
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def _mean_over_ranks(t):
    """Mean of a scalar tensor over the data-parallel ranks (the logged loss)."""
    world = _world()
    if world == 1:
        return t
    t = t.detach().clone()
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t / world


def train_one_epoch(model, loader, optimizer, scaler, epoch, device, config, writer, logger, normalizer=None):
    model.train()
    if normalizer is None:
        normalizer = ClipNormalizer(device=device)
    ssl_cfg = config["ssl"]
    train_cfg = config["training"]
    num_steps = len(loader)
    batch_size = train_cfg["batch_size"] * _world()      # global samples per step
    epoch_start = time.time()
    last_log = time.time()
    total_loss = 0.0
    for step, batch in enumerate(loader):
        clip = _to_clip(batch, device, normalizer)
        loss, pred, idx = train_step(model, clip, optimizer, scaler, ssl_cfg)
        loss = _mean_over_ranks(loss)
        total_loss += loss.item()
        if step % train_cfg["log_interval"] == 0 and step > 0:
            now = time.time()
            throughput = (train_cfg["log_interval"] * batch_size) / (now - last_log)
            eta = (now - epoch_start) / (step + 1) * (num_steps - step - 1)
            pred_std = masked_pred_std(pred, idx).item()
            logger.info(f"Epoch [{epoch}] [{step:4d}/{num_steps}] Loss: {loss.item():.4f} | Std: {pred_std:.3f} | "
                        f"Speed: {throughput:.1f} samples/s | Epoch ETA: {format_time(eta)}")
            last_log = now
            gstep = (epoch - 1) * num_steps + step
            writer.add_scalar("Train/Loss", loss.item(), gstep)
            writer.add_scalar("Train/Throughput", throughput, gstep)
    return total_loss / max(num_steps, 1), time.time() - epoch_start


def build_model(cfg, device="cuda"):
    """train_ssl_mae.py:143-144; `model.encoder` may name the build-defined
    "tiny_vit_small_variant" (BASELINE C3) instead of the reference's encoder."""
    make = ENCODERS[cfg.get("model", {}).get("encoder", "tiny_vit_21m_variant")]
    encoder = make(img_size=cfg["dataset"]["image_size"], use_checkpoint=True)
    return TinyVideoMAE(encoder, cfg).to(device)


def make_loader(ds, batch_size, num_workers=16, shuffle=True, sampler=None):
    """train_ssl_mae.py:154-161 (16 workers, pinned memory, prefetch 2) over the
    uint8-frame dataset (collate_frames); `sampler` (data parallel: a
    DistributedSampler) replaces the shuffle."""
    kw = {"prefetch_factor": 2} if num_workers > 0 else {}
    return torch.utils.data.DataLoader(ds, batch_size=batch_size, shuffle=shuffle and sampler is None,
                                       sampler=sampler, num_workers=num_workers, pin_memory=True,
                                       collate_fn=collate_frames, **kw)


class _RankZeroLogger:
    """Logger stand-in for ranks > 0 (the reference logs from its one process)."""

    def info(self, *a, **k):
        pass


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="configs/ssl_mae.yaml")
    ap.add_argument("--resume", default=None, help="training-state file written by a previous run")
    ap.add_argument("--max-steps", type=int, default=None, help="stop each epoch after this many steps")
    ap.add_argument("--arena", action="store_true",
                    help="device-memory arena instead of the caching allocator (ssl_mae_amd/arena.py; "
                         "lets the memory policy keep stage 0 resident at large batches); must be the "
                         "process's first CUDA use")
    args = ap.parse_args(argv)
    cfg = load_config(args.config)
    if args.arena:
        from . import arena
        arena.install(reserve_mib=8192 if int(os.environ.get("WORLD_SIZE", "1")) > 1 else None)
    rank, world = smdist.init_from_env()          # torchrun: one process per GPU (RCCL)
    set_seed(42)
    local = int(os.environ.get("LOCAL_RANK", "0")) if world > 1 else torch.cuda.current_device()
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if rank == 0:
        logger, log_dir = setup_logger(cfg["training"]["save_dir"])
        try:
            from torch.utils.tensorboard import SummaryWriter
            writer = SummaryWriter(log_dir=str(log_dir / "tensorboard"))
        except Exception:
            writer = NullWriter()
    else:
        logger, writer = _RankZeroLogger(), NullWriter()
    model = build_model(cfg, device)
    if rank > 0:
        # independent mask / frame-index streams per replica (rank 0 keeps the
        # reference's set_seed(42) streams; weights come from rank 0's broadcast)
        set_seed(42 + 1000 * rank)
    ds = LazyVideoMAEDataset(split_file=cfg["dataset"]["train_split"], clip_len=cfg["dataset"]["clip_len"],
                             stride=cfg["dataset"]["stride"], image_size=cfg["dataset"]["image_size"])
    sampler = torch.utils.data.DistributedSampler(ds, num_replicas=world, rank=rank, shuffle=True, seed=42) \
        if world > 1 else None
    loader = make_loader(ds, cfg["training"]["batch_size"], int(cfg["training"].get("num_workers", 16)),
                         sampler=sampler)
    if args.max_steps is not None:
        loader = _Limited(loader, args.max_steps)
    optimizer = FusedAdamW(model.parameters(), lr=float(cfg["training"]["lr"]),
                           weight_decay=float(cfg["training"].get("weight_decay", 0.05)))
    scaler = GradScaler("cuda")
    start = 1
    if args.resume:
        start = load_training_state(args.resume, model, optimizer, scaler)
        logger.info(f"Resumed from {args.resume} at epoch {start}")
    # rank 0's weights and buffers everywhere; bucketed gradient all-reduce hooked into
    # the backward (side stream) and the optimizer (world > 1)
    smdist.setup_data_parallel(model, optimizer, world)
    normalizer = ClipNormalizer(device=device)
    logger.info("=" * 50)
    logger.info(f"STARTING PRETRAINING | Total Epochs: {cfg['training']['epochs']}")
    logger.info(f"image size: {cfg['dataset']['image_size']} | Mask Ratio: {cfg['ssl']['mask_ratio']} | "
                f"clip_len: {cfg['dataset']['clip_len']}  | datasets: {cfg['dataset']['train_split']}")
    logger.info("=" * 50)
    t0 = time.time()
    save_dir = Path(cfg["training"]["save_dir"])
    epochs = cfg["training"]["epochs"]
    for epoch in range(start, epochs + 1):
        if sampler is not None:
            sampler.set_epoch(epoch)
        avg, dur = train_one_epoch(model, loader, optimizer, scaler, epoch, device, cfg, writer, logger,
                                   normalizer)
        total = time.time() - t0
        eta = total / (epoch - start + 1) * (epochs - epoch)
        logger.info("-" * 30)
        logger.info(f"==> Epoch {epoch} SUMMARY")
        logger.info(f"    Average Loss: {avg:.4f}")
        logger.info(f"    Training Time: {format_time(dur)}")
        logger.info(f"    Cumulative Time: {format_time(total)}")
        logger.info(f"    Total Training ETA: {format_time(eta)}")
        logger.info("-" * 30)
        if epoch % 10 == 0:
            rngs = gather_rng_states()            # every replica's streams (collective)
            if rank == 0:
                p = save_dir / f"encoder_ep{epoch}.pth"
                save_checkpoint(model.encoder.state_dict(), p)
                save_training_state(save_dir / "last_state.pth", model, optimizer, scaler, epoch, rngs)
                logger.info(f"Checkpoint saved to {p}")
            if world > 1:
                dist.barrier()
    return model


class _Limited:
    """First `n` batches of a loader (smoke runs of main())."""

    def __init__(self, loader, n):
        self.loader, self.n = loader, int(n)

    def __len__(self):
        return min(len(self.loader), self.n)

    def __iter__(self):
        for i, b in enumerate(self.loader):
            if i >= self.n:
                break
            yield b


if __name__ == "__main__":
    main()
