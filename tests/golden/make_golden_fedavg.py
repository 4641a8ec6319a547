"""Generate tests/golden/fedavg.npz by RUNNING the reference's FedAvg aggregation.

Build container only (the reference never travels).  Imports
src/federated/fed_loop.py and src/federated/comm_cost.py from /root/reference and
runs `fedavg_aggregate` on a small model that has every kind of state_dict entry
the reference distinguishes: fp32 weights and BN running stats, BN
num_batches_tracked (int64), an integer buffer, and a key one client lacks.
Output is data only: the global state, the client states, the weights, the
aggregated state, the comm-cost figures and the client schedule of run_fedavg.

    python tests/golden/make_golden_fedavg.py
"""
import importlib.util
import os
import random
import sys

import numpy as np
import torch
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))
REF_SRC = "/root/reference/src"


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


class Net(nn.Module):
    def __init__(self, extra=False):
        super().__init__()
        self.conv = nn.Conv2d(3, 8, 3, bias=False)
        self.bn = nn.BatchNorm2d(8)
        self.fc = nn.Linear(37, 13)   # odd sizes: ragged tails for the vector kernel
        self.register_buffer("idx", torch.arange(5, dtype=torch.int32))
        if extra:
            self.register_buffer("extra", torch.zeros(3))


def main():
    pkg = type(sys)("federated")
    pkg.__path__ = [os.path.join(REF_SRC, "federated")]
    sys.modules["federated"] = pkg
    _load("federated.comm_cost", os.path.join(REF_SRC, "federated", "comm_cost.py"))
    fl = _load("federated.fed_loop", os.path.join(REF_SRC, "federated", "fed_loop.py"))

    torch.manual_seed(7)
    glob = Net(extra=True)          # 'extra' missing from every client -> global value kept
    clients = [Net() for _ in range(3)]
    for i, c in enumerate(clients):
        with torch.no_grad():
            for p in c.parameters():
                p.normal_(0, 1.0 + i)
            c.bn.running_mean.normal_()
            c.bn.running_var.uniform_(0.5, 2.0)
            c.bn.num_batches_tracked.fill_(10 + 7 * i * (1 - i))   # 10, 10, -4 -> max 10 (non-first max too)
            c.idx.add_(i)
    clients[1].bn.num_batches_tracked.fill_(23)
    weights = [120.0, 37.0, 911.0]
    states = [{k: v.detach().clone() for k, v in c.state_dict().items()} for c in clients]
    g0 = {k: v.detach().clone() for k, v in glob.state_dict().items()}
    new_state = fl.fedavg_aggregate(glob, states, weights)
    comm_mb, model_mb = fl.estimate_comm_mb_per_round(new_state, num_clients_participating=3)

    rng = random.Random(42)
    sched = [rng.sample(list(range(5)), max(1, int(5 * 0.6))) for _ in range(4)]

    out = {"keys": np.array(list(g0.keys())), "weights": np.array(weights),
           "comm_mb": np.float64(comm_mb), "model_mb": np.float64(model_mb),
           "schedule_5c_f0.6_4r": np.array(sched, dtype=np.int64)}
    for k, v in g0.items():
        out[f"global/{k}"] = v.numpy()
    for i, s in enumerate(states):
        for k, v in s.items():
            out[f"client{i}/{k}"] = v.numpy()
    for k, v in new_state.items():
        out[f"out/{k}"] = v.numpy()
    np.savez(os.path.join(HERE, "fedavg.npz"), **out)
    print("wrote fedavg.npz:", len(out), "arrays")


if __name__ == "__main__":
    main()
