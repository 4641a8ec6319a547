"""Data parallelism: one process per GPU, gradients averaged over RCCL (xGMI).

The reference is single-device (train_ssl_mae.py:132); the north star shards the
batch over the 8 GPUs of a node.  Clips are independent apart from BatchNorm,
which keeps per-replica batch statistics (no SyncBN) — the natural DP semantic
of the reference's single-device BN.  Only the gradient exchange crosses GPUs:
the used range of the flat fp32 gradient buffer (20.45 M params, 78 MiB) is
all-reduced in large buckets (xGMI is point-to-point: a few big ring
collectives beat many small ones), SUM then scaled by 1/world on the GPU.
"""
import os

import torch
import torch.distributed as dist

from . import kernels as K

BUCKET_ELEMS = 8 * 1024 * 1024   # 32 MiB fp32 per collective


def init_from_env(backend=None):
    """Initialise torch.distributed from torchrun's env (RANK/WORLD_SIZE/MASTER_*)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1 or (dist.is_available() and dist.is_initialized()):
        return dist.get_rank() if dist.is_initialized() else 0, max(world, 1)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if backend == "nccl":
        torch.cuda.set_device(local)
    dist.init_process_group(backend=backend, rank=rank, world_size=world)
    return rank, world


def allreduce_flat(buf, world, group=None, bucket=BUCKET_ELEMS):
    """Average a flat fp32 tensor across ranks in place (bucketed SUM + 1/world)."""
    if world <= 1:
        return
    n = buf.numel()
    for s in range(0, n, bucket):
        dist.all_reduce(buf[s:s + bucket], op=dist.ReduceOp.SUM, group=group)
    if buf.is_cuda:
        K.scale_(buf, 1.0 / world)
    else:
        buf.mul_(1.0 / world)


class GradAllReduce:
    """FusedAdamW grad hook: average the used gradient range before the update."""

    def __init__(self, world, group=None):
        self.world = world
        self.group = group

    def __call__(self, flat):
        allreduce_flat(flat.grad[:flat.used_end], self.world, self.group)


def broadcast_params(flat, src=0, group=None):
    """Make every replica start from rank `src`'s weights (and BN buffers stay local)."""
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.broadcast(flat.data, src=src, group=group)
