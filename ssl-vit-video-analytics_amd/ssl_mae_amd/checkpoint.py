"""Full-MAE checkpoint and resume (SURVEY.md §5 "Checkpoint / resume", §8(f) rank 4).

The reference saves only the encoder every 10 epochs
(`src/train_ssl_mae.py:190-194` -> `utils.save_checkpoint`, `src/utils.py:73-77`):
no decoder, no optimizer state, no resume.  The build keeps that file unchanged
(`encoder_ep{N}.pth`, the keys `train_finetune` and FedAvg consume) and adds one
training-state file next to it with everything needed to continue bit-for-bit:

  model        full TinyVideoMAE state_dict (encoder + decoder + BN running stats)
  optimizer    FusedAdamW state (per-name exp_avg / exp_avg_sq, step, hyper-params)
  scaler       GradScaler shim state
  epoch        last finished epoch
  rng          torch CPU generator (drives the tube mask), device generators (seed
               AND state/offset, so torch device RNG use after a resume continues the
               stream), numpy / python RNG incl. python's cached gauss_next (drive the
               loader's frame-index choice)
  rng_ranks    the same record for every data-parallel rank (gathered at save time):
               each replica seeds its own streams (train_ssl_mae.main), so a resume
               restores rank r's streams on rank r -- the replicas keep drawing
               different tube masks and dropout / DropPath masks after a resume

Everything is a tensor / number / string, so `torch.load(..., weights_only=True)`
reads it back.
"""
import random
from pathlib import Path

import numpy as np
import torch


def _rng_state():
    np_state = np.random.get_state()
    py = random.getstate()
    st = {"torch_cpu": torch.get_rng_state(),
          "numpy_keys": torch.from_numpy(np_state[1].astype(np.int64)),
          "numpy_pos": int(np_state[2]), "numpy_has_gauss": int(np_state[3]), "numpy_gauss": float(np_state[4]),
          "python_version": int(py[0]), "python_state": torch.tensor(py[1], dtype=torch.int64),
          "python_has_gauss": int(py[2] is not None), "python_gauss": float(py[2]) if py[2] is not None else 0.0}
    if torch.cuda.is_available():
        st["cuda_seeds"] = torch.tensor([g.initial_seed() for g in torch.cuda.default_generators],
                                        dtype=torch.int64)
        st["cuda_states"] = [s.clone() for s in torch.cuda.get_rng_state_all()]
    return st


def _set_rng_state(st):
    torch.set_rng_state(st["torch_cpu"])
    np.random.set_state(("MT19937", st["numpy_keys"].numpy().astype(np.uint32), int(st["numpy_pos"]),
                         int(st["numpy_has_gauss"]), float(st["numpy_gauss"])))
    gauss = float(st["python_gauss"]) if int(st.get("python_has_gauss", 0)) else None
    random.setstate((int(st["python_version"]), tuple(int(v) for v in st["python_state"].tolist()), gauss))
    if "cuda_seeds" in st and torch.cuda.is_available():
        for g, s in zip(torch.cuda.default_generators, st["cuda_seeds"].tolist()):
            g.manual_seed(int(s))
        if "cuda_states" in st and len(st["cuda_states"]) == torch.cuda.device_count():
            torch.cuda.set_rng_state_all(st["cuda_states"])   # seed and offset


def _dist_world():
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def gather_rng_states():
    """Every rank's RNG record, in rank order (collective when data parallel: call it on
    all ranks, then let rank 0 write the file)."""
    st = _rng_state()
    rank, world = _dist_world()
    if world == 1:
        return [st]
    import torch.distributed as dist
    out = [None] * world
    dist.all_gather_object(out, st)
    return out


def save_training_state(path, model, optimizer, scaler, epoch, rng_states=None):
    """Write the full resumable state of an MAE run to `path`.  `rng_states`: the
    per-rank records from gather_rng_states() (default: this process only)."""
    path = Path(path)
    path.parent.mkdir(parents=True, exist_ok=True)
    rng_states = list(rng_states) if rng_states is not None else [_rng_state()]
    state = {"model": {k: v.detach().cpu() for k, v in model.state_dict().items()},
             "optimizer": _to_cpu(optimizer.state_dict()),
             "scaler": scaler.state_dict() if scaler is not None else {},
             "epoch": int(epoch),
             "forward_count": int(getattr(model, "_sm_fwd_count", 0)),
             "rng": rng_states[0],
             "rng_ranks": rng_states}
    tmp = path.with_suffix(path.suffix + ".tmp")
    torch.save(state, tmp)
    tmp.replace(path)
    return path


def load_training_state(path, model, optimizer, scaler=None):
    """Restore a state written by save_training_state; returns the epoch to start
    from (last finished epoch + 1)."""
    state = torch.load(path, map_location="cpu", weights_only=True)
    model.load_state_dict(state["model"], strict=True)
    from .mae_vit_adapter import ensure_flat
    from .functions import Mode
    ensure_flat(model, Mode(False))       # parameters live in the flat buffer before the optimizer state
    optimizer.load_state_dict(state["optimizer"])
    if scaler is not None and state.get("scaler"):
        scaler.load_state_dict(state["scaler"])
    model._sm_fwd_count = int(state.get("forward_count", 0))
    restore_rank_rng(state)
    return int(state["epoch"]) + 1


def restore_rank_rng(state):
    """This rank's streams: rng_ranks[rank] when the file was written by a run of the
    same world size; otherwise rank 0's record, re-seeded on ranks > 0 with the rank
    mixed in (a file from a single-process run, or another world size), so the
    replicas still draw independent masks."""
    rank, world = _dist_world()
    ranks = state.get("rng_ranks")
    if ranks is not None and len(ranks) == world:
        _set_rng_state(ranks[rank])
        return
    _set_rng_state(state["rng"])
    if rank > 0:
        from .utils import set_seed
        base = int(torch.randint(0, 2 ** 30, (1,)).item())
        set_seed(base + 1000 * rank)


def _to_cpu(x):
    if torch.is_tensor(x):
        return x.detach().cpu()
    if isinstance(x, dict):
        return {k: _to_cpu(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return type(x)(_to_cpu(v) for v in x)
    return x
