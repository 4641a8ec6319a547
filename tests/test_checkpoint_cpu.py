"""Resume RNG state (ssl_mae_amd/checkpoint.py): every host stream the driver and the
loader draw from continues exactly after a save/restore, including python's cached
second Box-Muller normal (random.gauss's gauss_next)."""
import random

import numpy as np
import torch


def test_rng_state_round_trip_host_streams(tmp_path):
    from ssl_mae_amd.checkpoint import _rng_state, _set_rng_state
    random.seed(7)
    np.random.seed(7)
    torch.manual_seed(7)
    random.gauss(0.0, 1.0)            # leaves gauss_next cached
    np.random.standard_normal()       # leaves numpy's cached gauss
    st = _rng_state()
    torch.save(st, tmp_path / "rng.pth")
    a = (random.gauss(0.0, 1.0), random.random(), float(np.random.standard_normal()), torch.rand(3).tolist())
    random.seed(99)
    np.random.seed(99)
    torch.manual_seed(99)
    _set_rng_state(torch.load(tmp_path / "rng.pth", weights_only=True))
    b = (random.gauss(0.0, 1.0), random.random(), float(np.random.standard_normal()), torch.rand(3).tolist())
    assert a == b


def _dp_rng_worker(rank, world, port, path, q):
    import os
    import sys
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [here, os.path.join(here, "ssl-vit-video-analytics_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    from ssl_mae_amd.checkpoint import gather_rng_states, restore_rank_rng
    from ssl_mae_amd.utils import set_seed
    dist.init_process_group("gloo", rank=rank, world_size=world)
    set_seed(42 + 1000 * rank)                    # train_ssl_mae.main's per-replica streams
    torch.rand(100)
    rngs = gather_rng_states()
    if rank == 0:
        torch.save({"rng": rngs[0], "rng_ranks": rngs}, path)
        torch.save({"rng": rngs[0]}, path + ".single")     # a single-process file
    expect = torch.rand(2, 784)                   # the tube-mask noise the next step draws
    dist.barrier()
    set_seed(7)                                   # scramble, then resume
    restore_rank_rng(torch.load(path, weights_only=True))
    got = torch.rand(2, 784)
    restore_rank_rng(torch.load(path + ".single", weights_only=True))
    single = torch.rand(2, 784)
    q.put((rank, expect, got, single))
    dist.barrier()
    dist.destroy_process_group()


def test_data_parallel_resume_restores_each_ranks_streams(tmp_path):
    """a resume under data parallelism restores rank r's own RNG streams
    (gathered at save time), so replicas keep drawing different tube masks; a file
    holding one record re-seeds ranks > 0 with the rank mixed in."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    path = str(tmp_path / "state.pth")
    procs = [ctx.Process(target=_dp_rng_worker, args=(r, 2, port, path, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (e, g, s1)) for r, e, g, s1 in (q.get(timeout=120) for _ in range(2)))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for r in (0, 1):
        assert torch.equal(res[r][0], res[r][1]), r          # each rank continues its own stream
    assert not torch.equal(res[0][1], res[1][1])             # replicas stay independent
    assert not torch.equal(res[0][2], res[1][2])             # also from a single-record file
    assert torch.equal(res[0][2], res[0][0])                 # rank 0 keeps the saved record
