"""The drop-in driver, data parallel: `main(["--max-steps", "1"])` on two ranks
sharing the card over gloo (CUDA tensors; RCCL needs one GPU per rank).  Each rank
reads its own shard of the split (DistributedSampler), so the ranks see different
clips; after the step every replica must hold identical parameters (rank 0's
broadcast start + the bucketed all-reduce of the gradients inside the backward),
while BatchNorm running statistics stay per replica.  Only rank 0 writes the
checkpoint files.  Reference: src/train_ssl_mae.py:129-194 (single device, :132)."""
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _worker(rank, world, port, root, cfg_path, q):
    import sys
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [here, os.path.join(here, "ssl-vit-video-analytics_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0")
    os.chdir(root)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)    # main() keeps an existing group
    torch.cuda.set_device(0)
    from ssl_mae_amd import train_ssl_mae as TR
    seen = []
    orig = TR.train_step

    def spy(model, clip, *a, **k):
        seen.append(float(clip.double().sum()))
        return orig(model, clip, *a, **k)
    TR.train_step = spy
    model = TR.main(["--config", cfg_path, "--max-steps", "1"])
    params = {n: p.detach().cpu().numpy().copy() for n, p in model.named_parameters()}
    bufs = {n: b.detach().cpu().numpy().copy() for n, b in model.named_buffers() if "running_mean" in n}
    q.put((rank, params, bufs, seen))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(600)
def test_main_data_parallel_world2_replicas_identical(tmp_path):
    import torch.multiprocessing as mp
    from test_driver_gpu import _config, _dataset
    split = _dataset(tmp_path, n_videos=4)
    cfg = _config(tmp_path, split, 10)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, str(tmp_path), str(cfg), q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        r, params, bufs, seen = q.get(timeout=540)
        res[r] = (params, bufs, seen)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    p0, b0, s0 = res[0]
    p1, b1, s1 = res[1]
    assert len(s0) == len(s1) == 10 and s0 != s1            # one step per epoch, different shards
    for n in p0:
        assert np.array_equal(p0[n], p1[n]), n               # replicas identical after 10 steps
    assert any(not np.array_equal(b0[n], b1[n]) for n in b0)   # per-replica BN statistics
    save_dir = tmp_path / "results" / "tinymae_test"
    assert (save_dir / "encoder_ep10.pth").exists() and (save_dir / "last_state.pth").exists()
