"""CPU ORACLE — TEST INFRASTRUCTURE ONLY.

numpy restatement of the reference's FedAvg aggregation and communication
accounting.  Only `tests/` may import it, as the checker; the product path
(ssl_mae_amd.federated) never does.

Pinned by tests/golden/fedavg.npz, produced by RUNNING the reference's
`fedavg_aggregate` / `estimate_comm_mb_per_round` in the build container
(tests/golden/make_golden_fedavg.py; checked by tests/test_fedavg_cpu.py).

What it follows (reference file:line, relative to the reference repo root):
  fedavg_aggregate            src/federated/fed_loop.py:14-62
      float entries           :45-49  acc = 0; acc += x.to(f32) * (w / total_w),
                                      product and sum each rounded to fp32, client order
      num_batches_tracked     :52-55  elementwise max over clients
      other non-float         :57-58  copied from the first client
      key missing in a client :40-42  the global model's value
  model_size_bytes            src/federated/comm_cost.py:4-10
  estimate_comm_mb_per_round  src/federated/comm_cost.py:17-26 (2 N model bytes)
  client sampling             src/federated/fed_loop.py:85,90-91
                              (random.Random(42).sample per round)
"""
import random

import numpy as np


def check_inputs(client_states, client_weights):
    """fed_loop.py:24-31 error conditions."""
    if len(client_states) == 0:
        raise RuntimeError("[ERROR] No client states provided for aggregation.")
    if len(client_states) != len(client_weights):
        raise RuntimeError("[ERROR] client_states and client_weights length mismatch.")
    total_w = float(sum(client_weights))
    if total_w <= 0:
        raise RuntimeError("[ERROR] total client weight must be > 0.")
    return total_w


def weighted_sum(arrays, weights):
    """fed_loop.py:46-49 for one fp32 entry: sequential, separately rounded."""
    total_w = float(sum(weights))
    acc = np.zeros_like(np.asarray(arrays[0], dtype=np.float32))
    for x, w in zip(arrays, weights):
        s = np.float32(float(w) / total_w)
        acc = (acc + (np.asarray(x, dtype=np.float32) * s).astype(np.float32)).astype(np.float32)
    return acc


def fedavg_aggregate(global_state, client_states, client_weights):
    """fed_loop.py:14-62 over dicts of numpy arrays -> new state dict."""
    check_inputs(client_states, client_weights)
    out = {}
    for k, g in global_state.items():
        if any(k not in cs for cs in client_states):
            out[k] = np.array(g)
        elif np.issubdtype(np.asarray(g).dtype, np.floating):
            out[k] = weighted_sum([cs[k] for cs in client_states], client_weights)
        elif "num_batches_tracked" in k:
            out[k] = np.max(np.stack([np.asarray(cs[k], dtype=np.int64) for cs in client_states]), axis=0)
        else:
            out[k] = np.array(client_states[0][k])
    return out


def model_size_bytes(state):
    return int(sum(np.asarray(v).size * np.asarray(v).dtype.itemsize for v in state.values()))


def estimate_comm_mb_per_round(state, num_clients_participating):
    size_b = model_size_bytes(state)
    return float(2 * int(num_clients_participating) * size_b) / 2 ** 20, float(size_b) / 2 ** 20


def client_schedule(num_clients, rounds, client_fraction=1.0):
    """fed_loop.py:85,90-91: the clients selected in each round."""
    rng = random.Random(42)
    m = max(1, int(num_clients * float(client_fraction)))
    return [rng.sample(list(range(num_clients)), m) for _ in range(int(rounds))]
