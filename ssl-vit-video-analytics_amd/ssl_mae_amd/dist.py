"""Data parallelism: one process per GPU, gradients averaged over RCCL (xGMI),
overlapped with the backward.

The reference is single-device (train_ssl_mae.py:132); the north star shards the
batch over the 8 GPUs of a node.  Clips are independent apart from BatchNorm,
which keeps per-replica batch statistics (no SyncBN) — the natural DP semantic
of the reference's single-device BN.  Only the gradient exchange crosses GPUs.

Layout: the used range of the flat fp32 gradient buffer (20.45 M params,
78 MiB) is ordered the way the backward produces gradients (optim.FlatParams,
mae_vit_adapter.gradient_order) and cut into ~24 MiB buckets of whole parameters
(SURVEY.md §8(e)).  Every fused backward group ends with `FlatParams.done(...)`;
when the last parameter of a bucket is written, `OverlappedGradAllReduce`
records an event on the compute stream and, on its own side HIP stream, waits
for it, all-reduces the bucket (SUM, RCCL ring over xGMI; large buckets because
the links are point-to-point and per-link bound) and scales it by 1/world.  The
decoder's buckets are therefore reduced while the encoder's backward still runs.
Before AdamW, `finish()` launches any bucket not yet launched and makes the compute
stream wait for the side stream.  On CPU (gloo tests) the same control flow runs
synchronously.
"""
import os

import torch
import torch.distributed as dist

from . import ops as K    # every kernel launch through the torch.ops.ssl_mae dispatcher

BUCKET_ELEMS = 6 * 1024 * 1024   # 24 MiB fp32 per collective


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


def _scale(buf, a):
    if buf.is_cuda:
        K.scale_(buf, a)
    else:
        buf.mul_(a)


def allreduce_flat(buf, world, group=None, bucket=BUCKET_ELEMS):
    """Average a flat fp32 tensor across ranks in place (bucketed SUM + 1/world)."""
    if world <= 1:
        return
    n = buf.numel()
    for s in range(0, n, bucket):
        dist.all_reduce(buf[s:s + bucket], op=dist.ReduceOp.SUM, group=group)
    _scale(buf, 1.0 / world)


class OverlappedGradAllReduce:
    """Bucketed gradient all-reduce launched from the backward (see module doc).

    Register with `attach(flat, optimizer)`; `launched` records the bucket order of
    the last step (tests check that buckets start before the backward ends)."""

    def __init__(self, world, group=None, bucket_elems=BUCKET_ELEMS):
        self.world = world
        self.group = group
        self.bucket_elems = bucket_elems
        self.flat = None
        self.side = None
        self.launched = []
        self.trace = None          # optional callable(event) for tests

    def attach(self, flat, optimizer):
        self.flat = flat
        flat.make_buckets(self.bucket_elems)
        flat.ready_hooks.append(self.bucket_ready)
        optimizer.grad_hooks.append(self.finish)
        if flat.grad.is_cuda:
            self.side = torch.cuda.Stream(device=flat.grad.device)
        return self

    def bucket_ready(self, b):
        if b in self.launched:
            return
        self.launched.append(b)
        s, e = self.flat.bucket_ranges[b]
        buf = self.flat.grad[s:e]
        if self.trace is not None:
            self.trace(("launch", b))
        if self.side is None:
            dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.group)
            _scale(buf, 1.0 / self.world)
            return
        ready = torch.cuda.Event()
        ready.record()                                   # compute stream: bucket's grads written
        with torch.cuda.stream(self.side):
            self.side.wait_event(ready)
            dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.group)
            _scale(buf, 1.0 / self.world)

    def finish(self, flat):
        """FusedAdamW grad hook: every bucket reduced before the update."""
        for b in range(len(flat.bucket_ranges)):
            if b not in self.launched:
                self.bucket_ready(b)
        if self.side is not None:
            torch.cuda.current_stream().wait_stream(self.side)
        if self.trace is not None:
            self.trace(("finish", list(self.launched)))
        self.launched = []


class GradAllReduce:
    """FusedAdamW grad hook without overlap: average the used gradient range after
    the backward (kept for A/B measurements)."""

    def __init__(self, world, group=None):
        self.world = world
        self.group = group

    def __call__(self, flat):
        allreduce_flat(flat.grad[:flat.used_end], self.world, self.group)


def broadcast_params(flat, src=0, group=None):
    """Make every replica start from rank `src`'s weights."""
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.broadcast(flat.data, src=src, group=group)


def broadcast_buffers(module, src=0, group=None):
    """BatchNorm running statistics (and any other buffers) from rank `src`."""
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        for b in module.buffers():
            dist.broadcast(b, src=src, group=group)


def setup_data_parallel(model, optimizer, world, group=None, bucket_elems=BUCKET_ELEMS):
    """One call per rank after building the model and its FusedAdamW: lays the
    parameters into the flat buffer, broadcasts rank 0's weights and buffers, and
    hooks the overlapped bucketed all-reduce into the backward and the optimizer."""
    from .functions import Mode
    from .mae_vit_adapter import ensure_flat
    flat = getattr(model, "_sm_flat", None) or ensure_flat(model, Mode(False))
    broadcast_params(flat, 0, group)
    broadcast_buffers(model, 0, group)
    if world <= 1:
        return None
    return OverlappedGradAllReduce(world, group, bucket_elems).attach(flat, optimizer)
