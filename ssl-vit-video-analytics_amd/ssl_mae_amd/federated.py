"""FedAvg aggregation on MI355X (reference: src/federated/fed_loop.py, comm_cost.py).

Same API as the reference module: `fedavg_aggregate(global_model, client_states,
client_weights)`, `run_fedavg(...)`, `estimate_comm_mb_per_round(state, n)`,
`model_size_bytes`, `bytes_to_mb`, with the same error conditions and the same
per-key rules (fed_loop.py:38-58):

  * floating-point entries: weighted average, accumulated in client order with
    separately rounded products and sums — one HIP launch over ONE flat fp32
    buffer per client (sm_fedavg_weighted_sum), bit-identical to the reference;
  * `num_batches_tracked`: elementwise max over clients (sm_fedavg_counters_max);
  * other integer entries: copied from the first client;
  * a key missing from any client: the global model's value.

Difference from the reference: it aggregates on the CPU "to avoid GPU memory
spikes" (fed_loop.py:22); here the model is ~80 MiB and HBM is 288 GB, so the
client states are staged into device buffers and the result stays on the global
model's device.  The flattening (one torch.cat per client) is data movement; the
arithmetic is the HIP kernel — there is no CPU arithmetic path.

Multi-GPU (BASELINE config C5, 4 clients on 4 GPUs): `fedavg_allgather` makes
every rank one client.  Each rank's flat fp32 state is all-gathered over RCCL
(one collective per round, (N-1) x 80 MiB per rank over xGMI ~ 2 ms at N=4),
then every rank runs the same weighted-sum kernel in rank order, so every
replica holds exactly the reference's aggregate (an all-reduce SUM would be
cheaper but its ring order breaks bit-exactness, and the exchange happens once
per round).  Counters take a MAX all-reduce; other integer buffers come from
rank 0 (the "first client").
"""
import random

import torch
import torch.distributed as dist

from . import ops as K    # every kernel launch through the torch.ops.ssl_mae dispatcher


def _is_float_tensor(t):
    return torch.is_tensor(t) and torch.is_floating_point(t)


def _check(client_states, client_weights):
    # fed_loop.py:24-31
    if len(client_states) == 0:
        raise RuntimeError("[ERROR] No client states provided for aggregation.")
    if len(client_states) != len(client_weights):
        raise RuntimeError("[ERROR] client_states and client_weights length mismatch.")
    total_w = float(sum(client_weights))
    if total_w <= 0:
        raise RuntimeError("[ERROR] total client weight must be > 0.")
    return total_w


def _norm_weights(client_weights, total_w):
    # torch multiplies an fp32 tensor by the Python double w / total_w in fp32
    # (the scalar is rounded to fp32 first): the kernel takes those fp32 values.
    return [float(torch.tensor(float(w) / total_w, dtype=torch.float32)) for w in client_weights]


def _device_of(global_model, global_state):
    for v in global_state.values():
        if torch.is_tensor(v):
            return v.device
    return next(global_model.parameters()).device


def _flat(tensors, device, dtype):
    return torch.cat([t.detach().reshape(-1).to(device=device, dtype=dtype) for t in tensors])


def fedavg_aggregate(global_model, client_states, client_weights):
    """fed_loop.py:14-62.  Aggregates, loads the result into `global_model`
    (strict) and returns the new state dict (tensors on the model's device)."""
    total_w = _check(client_states, client_weights)
    global_state = global_model.state_dict()
    device = _device_of(global_model, global_state)
    if device.type != "cuda":
        raise RuntimeError("ssl_mae_amd FedAvg runs on the GPU only (move the global model with .to('cuda'))")

    new_state = {}
    float_keys, count_keys = [], []
    norm = _norm_weights(client_weights, total_w)
    for k, g in global_state.items():
        if any(k not in cs for cs in client_states):
            new_state[k] = g.detach().clone()
        elif _is_float_tensor(g):
            if g.dtype == torch.float32:
                float_keys.append(k)
            else:
                # fp16 / bf16 / fp64 entries (not produced by the MAE models): the
                # reference's per-key accumulation in the entry's own dtype
                # (fed_loop.py:46-49), as device tensor ops on the global model's GPU.
                acc = torch.zeros_like(g.detach())
                for cs, w in zip(client_states, client_weights):
                    acc += cs[k].detach().to(device=device, dtype=acc.dtype) * (float(w) / total_w)
                new_state[k] = acc
        elif "num_batches_tracked" in k:
            count_keys.append(k)
        else:
            new_state[k] = client_states[0][k].detach().to(device).clone()

    if float_keys:
        bufs = [_flat([cs[k] for k in float_keys], device, torch.float32) for cs in client_states]
        out = K.fedavg_weighted_sum(bufs, norm)
        _unflat(out, float_keys, global_state, new_state)
    if count_keys:
        bufs = [_flat([cs[k] for k in count_keys], device, torch.int64) for cs in client_states]
        out = K.fedavg_counters_max(bufs)
        _unflat(out, count_keys, global_state, new_state)

    new_state = {k: new_state[k] for k in global_state}   # reference key order
    global_model.load_state_dict(new_state, strict=True)
    return new_state


def _unflat(flat, keys, like, dst):
    off = 0
    for k in keys:
        n = like[k].numel()
        dst[k] = flat[off:off + n].view(like[k].shape)
        off += n


# ------------------------------------------------------------------ multi-GPU (C5)
def fedavg_allgather(model, weight, group=None, combine=None):
    """Every rank is one client: replace `model`'s state on every rank with the
    FedAvg of all ranks' states (rank order = client order), in place.

    `combine(bufs, norm_weights) -> flat` is the weighted sum; it defaults to the
    HIP kernel (device tensors required).  Returns the total client weight."""
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    state = model.state_dict()
    device = _device_of(model, state)
    float_keys = [k for k, v in state.items() if _is_float_tensor(v)]
    count_keys = [k for k, v in state.items() if not _is_float_tensor(v) and "num_batches_tracked" in k]
    other_keys = [k for k, v in state.items() if not _is_float_tensor(v) and "num_batches_tracked" not in k]
    for k in float_keys:
        if state[k].dtype != torch.float32:
            raise RuntimeError(f"fedavg_allgather aggregates fp32 state only; {k} is {state[k].dtype} "
                               "(use fedavg_aggregate, which follows the reference for any float dtype)")

    w = torch.tensor([float(weight)], dtype=torch.float64, device=device)
    ws = [torch.empty_like(w) for _ in range(world)]
    if world > 1:
        dist.all_gather(ws, w, group=group)
    else:
        ws = [w]
    client_weights = [float(x.item()) for x in ws]
    total_w = _check([None] * world, client_weights)
    norm = _norm_weights(client_weights, total_w)

    if combine is None:
        combine = K.fedavg_weighted_sum
    new_state = {}
    if float_keys:
        mine = _flat([state[k] for k in float_keys], device, torch.float32)
        if world > 1:
            bufs = [torch.empty_like(mine) for _ in range(world)]
            dist.all_gather(bufs, mine, group=group)
        else:
            bufs = [mine]
        _unflat(combine(bufs, norm), float_keys, state, new_state)
    if count_keys:
        cnt = _flat([state[k] for k in count_keys], device, torch.int64)
        if world > 1:
            dist.all_reduce(cnt, op=dist.ReduceOp.MAX, group=group)
        _unflat(cnt, count_keys, state, new_state)
    if other_keys:
        oth = [state[k].detach().clone() for k in other_keys]
        if world > 1:
            src = dist.get_global_rank(group, 0) if group is not None else 0
            for t in oth:
                dist.broadcast(t, src=src, group=group)
        new_state.update(dict(zip(other_keys, oth)))
    model.load_state_dict({k: new_state[k] for k in state}, strict=True)
    return total_w


# ------------------------------------------------------------------ comm accounting (comm_cost.py)
def model_size_bytes(state_dict):
    """comm_cost.py:4-10."""
    return int(sum(v.numel() * v.element_size() for v in state_dict.values() if torch.is_tensor(v)))


def bytes_to_mb(x):
    """comm_cost.py:13-14."""
    return float(x) / (1024.0 * 1024.0)


def estimate_comm_mb_per_round(global_state, num_clients_participating):
    """comm_cost.py:17-26: broadcast + upload = 2 N model bytes."""
    size_b = model_size_bytes(global_state)
    return bytes_to_mb(int(2 * int(num_clients_participating) * size_b)), bytes_to_mb(size_b)


# ------------------------------------------------------------------ host loop (fed_loop.py:65-150)
def run_fedavg(global_model, client_models, client_loaders, client_sizes, evaluate_fn, device, rounds=10,
               client_fraction=1.0, amp=True, log_f=None):
    """fed_loop.py:65-150: each round samples clients with random.Random(42),
    broadcasts the global weights, runs client_loaders[cid]["update_fn"](model),
    aggregates with fedavg_aggregate and evaluates.  Returns the per-round records."""
    num_clients = len(client_models)
    rng = random.Random(42)
    records = []

    def log(msg):
        print(msg)
        if log_f:
            log_f.write(msg + "\n")
            log_f.flush()

    for r in range(1, int(rounds) + 1):
        m = max(1, int(num_clients * float(client_fraction)))
        selected = rng.sample(list(range(num_clients)), m)
        log(f"[INFO] Round {r}/{rounds} selected_clients={selected}")
        g = {k: v.detach().clone() for k, v in global_model.state_dict().items()}
        for cid in selected:
            client_models[cid].load_state_dict(g, strict=True)
        states, weights, losses = [], [], []
        for cid in selected:
            losses.append(float(client_loaders[cid]["update_fn"](client_models[cid])))
            states.append({k: v.detach() for k, v in client_models[cid].state_dict().items()})
            weights.append(float(client_sizes[cid]))
        new_state = fedavg_aggregate(global_model, states, weights)
        comm_total_mb, model_mb = estimate_comm_mb_per_round(new_state, num_clients_participating=len(selected))
        top1, top5 = evaluate_fn(global_model)
        rec = {"round": r, "val_top1": float(top1), "val_top5": float(top5),
               "avg_local_loss": float(sum(losses) / max(1, len(losses))), "clients": int(len(selected)),
               "model_mb": float(model_mb), "comm_mb_round": float(comm_total_mb)}
        records.append(rec)
        log(f"[INFO] Round {r} val_top1={top1:.4f} val_top5={top5:.4f} "
            f"avg_local_loss={rec['avg_local_loss']:.4f} comm_mb={comm_total_mb:.2f}")
    return records
