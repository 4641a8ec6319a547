"""FedAvg (BASELINE config C5) on CPU: no GPU needed.

* the numpy oracle (oracle/fedavg_oracle.py) reproduces the reference's own
  `fedavg_aggregate` output bit for bit on tests/golden/fedavg.npz (produced by
  running src/federated/fed_loop.py; make_golden_fedavg.py), plus its comm-cost
  figures and run_fedavg's client schedule;
* the host mirror's weight normalisation (fp32 rounding of w / total_w) is what
  torch does to `tensor * python_float` — the kernel's scalar contract;
* the multi-GPU path `fedavg_allgather` over 2 gloo ranks (the weighted sum
  supplied by the oracle, since the HIP kernel needs a GPU) equals the oracle's
  aggregate of both ranks' states, counters by max, ints from rank 0.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import GOLDEN


def _golden():
    z = np.load(os.path.join(GOLDEN, "fedavg.npz"))
    keys = [str(k) for k in z["keys"]]
    g = {k: z[f"global/{k}"] for k in keys}
    clients = []
    i = 0
    while f"client{i}/conv.weight" in z:
        clients.append({k[len(f"client{i}/"):]: z[k] for k in z.files if k.startswith(f"client{i}/")})
        i += 1
    out = {k: z[f"out/{k}"] for k in keys}
    return z, g, clients, [float(w) for w in z["weights"]], out


def test_oracle_matches_reference_fedavg_bit_exact():
    from oracle import fedavg_oracle as O
    z, g, clients, w, ref = _golden()
    got = O.fedavg_aggregate(g, clients, w)
    assert list(got) == list(ref)
    for k in ref:
        assert got[k].dtype == ref[k].dtype, k
        assert np.array_equal(got[k], ref[k]), k
    # the rules the golden exercises
    assert np.array_equal(ref["extra"], g["extra"])                       # key missing in clients
    assert int(ref["bn.num_batches_tracked"]) == 23                        # max, not first client
    assert np.array_equal(ref["idx"], clients[0]["idx"])                   # int copied from client 0


def test_oracle_comm_cost_and_schedule_match_reference():
    from oracle import fedavg_oracle as O
    z, g, clients, w, ref = _golden()
    comm, model = O.estimate_comm_mb_per_round(ref, 3)
    assert comm == float(z["comm_mb"]) and model == float(z["model_mb"])
    assert np.array_equal(np.array(O.client_schedule(5, 4, 0.6)), z["schedule_5c_f0.6_4r"])


def test_host_comm_cost_matches_reference():
    from ssl_mae_amd import federated as F
    z, g, clients, w, ref = _golden()
    st = {k: torch.from_numpy(v) for k, v in ref.items()}
    assert F.estimate_comm_mb_per_round(st, 3) == (float(z["comm_mb"]), float(z["model_mb"]))


def test_oracle_error_conditions():
    from oracle import fedavg_oracle as O
    with pytest.raises(RuntimeError, match="No client states"):
        O.check_inputs([], [])
    with pytest.raises(RuntimeError, match="length mismatch"):
        O.check_inputs([{}], [1.0, 2.0])
    with pytest.raises(RuntimeError, match="must be > 0"):
        O.check_inputs([{}], [0.0])


def test_host_error_conditions_match_reference():
    from ssl_mae_amd import federated as F
    m = torch.nn.Linear(2, 2)
    with pytest.raises(RuntimeError, match="No client states"):
        F.fedavg_aggregate(m, [], [])
    with pytest.raises(RuntimeError, match="length mismatch"):
        F.fedavg_aggregate(m, [m.state_dict()], [1.0, 2.0])
    with pytest.raises(RuntimeError, match="must be > 0"):
        F.fedavg_aggregate(m, [m.state_dict()], [0.0])
    with pytest.raises(RuntimeError, match="GPU only"):          # no CPU arithmetic path
        F.fedavg_aggregate(m, [m.state_dict()], [1.0])


def test_weight_rounding_is_torchs_scalar_rule():
    """torch computes fp32_tensor * python_float with the scalar rounded to fp32."""
    from ssl_mae_amd import federated as F
    rng = np.random.default_rng(3)
    x = torch.from_numpy(rng.standard_normal(4099).astype(np.float32))
    for w in ([120.0, 37.0, 911.0], [1.0, 3.0], [0.1, 0.7, 0.2, 1e-3]):
        tot = float(sum(w))
        for wi, ni in zip(w, F._norm_weights(w, tot)):
            a = (x * (float(wi) / tot)).numpy()
            b = (x.numpy() * np.float32(ni)).astype(np.float32)
            assert np.array_equal(a, b)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


class _Net(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.fc = torch.nn.Linear(19, 7)
        self.bn = torch.nn.BatchNorm1d(7)
        self.register_buffer("idx", torch.arange(3, dtype=torch.int32))


def _worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "ssl-vit-video-analytics_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from oracle import fedavg_oracle as O
    from ssl_mae_amd import dist as smdist
    from ssl_mae_amd import federated as F
    smdist.init_from_env(backend="gloo")
    torch.manual_seed(100 + rank)
    net = _Net()
    with torch.no_grad():
        net.bn.running_mean.normal_()
        net.bn.num_batches_tracked.fill_(5 + 9 * rank)
        net.idx.add_(10 * rank)
    before = {k: v.detach().clone().numpy() for k, v in net.state_dict().items()}

    def combine(bufs, norm):
        acc = np.zeros(bufs[0].numel(), np.float32)
        for b, s in zip(bufs, norm):
            acc = (acc + (b.numpy() * np.float32(s)).astype(np.float32)).astype(np.float32)
        return torch.from_numpy(acc)

    weight = [30.0, 70.0][rank]
    tot = F.fedavg_allgather(net, weight, combine=combine)
    after = {k: v.detach().clone().numpy() for k, v in net.state_dict().items()}
    q.put((rank, tot, before, after))
    import torch.distributed as dist
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_gloo_world2_fedavg_allgather():
    from oracle import fedavg_oracle as O
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, tot, before, after = q.get(timeout=240)
        res[r] = (tot, before, after)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    expect = O.fedavg_aggregate(res[0][1], [res[0][1], res[1][1]], [30.0, 70.0])
    for r in range(world):
        assert res[r][0] == 100.0
        for k, v in expect.items():
            assert np.array_equal(res[r][2][k], v), (r, k)
    assert int(expect["bn.num_batches_tracked"]) == 14
