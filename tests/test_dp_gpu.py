"""Data-parallel step on the GPU: two ranks sharing the card over gloo (CUDA
tensors; RCCL needs one GPU per rank, which this box does not have).  Runs the
production path end to end -- the fused HIP backward calling FlatParams.done(),
bucket all-reduces enqueued on the side HIP stream behind a compute-stream event,
finish() joining the streams before sm_adamw -- and checks the reduced gradient
equals the mean of the two ranks' un-reduced gradients bit for bit, and that both
replicas hold identical parameters after the step."""
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _cfg():
    return {"dataset": {"clip_len": 2, "image_size": 32, "stride": 4, "train_split": "-"},
            "model": {"decoder_embed_dim": 384, "decoder_depth": 2, "decoder_num_heads": 6},
            "ssl": {"mask_ratio": 0.75, "norm_pix_loss": True},
            "training": {"batch_size": 1, "lr": 5e-4, "log_interval": 20}}


def _model(cfg):
    from ssl_mae_amd import parity_mode
    from ssl_mae_amd.init_rule import apply_rule
    from ssl_mae_amd.mae_vit_adapter import TinyVideoMAE
    from ssl_mae_amd.tiny_vit import tiny_vit_21m_variant
    m = TinyVideoMAE(tiny_vit_21m_variant(img_size=32), cfg)
    apply_rule(m)
    return parity_mode(m).cuda().train()


def _worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "ssl-vit-video-analytics_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0")
    import torch.distributed as dist
    from ssl_mae_amd import dist as smdist
    from ssl_mae_amd.init_rule import synthetic_clip
    from ssl_mae_amd.optim import FusedAdamW, GradScaler
    from ssl_mae_amd.train_ssl_mae import train_step
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    cfg = _cfg()
    clip = torch.from_numpy(synthetic_clip(1, 2, 32, seed=50 + rank)).cuda()
    # 1) this rank's own gradient (no data parallelism)
    solo = _model(cfg)
    opt_s = FusedAdamW(solo.parameters(), lr=5e-4, weight_decay=0.05)
    torch.manual_seed(7 + rank)
    train_step(solo, clip, opt_s, GradScaler(), cfg["ssl"], bf16=True)
    g_solo = solo._sm_flat.grad[:solo._sm_flat.used_end].clone()
    # 2) the data-parallel step (overlapped bucketed all-reduce)
    model = _model(cfg)
    opt = FusedAdamW(model.parameters(), lr=5e-4, weight_decay=0.05)
    red = smdist.setup_data_parallel(model, opt, world, bucket_elems=1 << 20)
    events = []
    red.trace = events.append
    torch.manual_seed(7 + rank)
    loss, _, _ = train_step(model, clip, opt, GradScaler(), cfg["ssl"], bf16=True)
    torch.cuda.synchronize()
    flat = model._sm_flat
    gs = [torch.empty_like(g_solo) for _ in range(world)]
    dist.all_gather(gs, g_solo)
    mean = (gs[0] + gs[1]) * 0.5
    q.put((rank, torch.equal(flat.grad[:flat.used_end], mean), len(flat.bucket_ranges), events,
           flat.data.cpu().numpy().copy(), float(loss)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_data_parallel_overlapped_step_world2():
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        r, same, nb, events, data, loss = q.get(timeout=240)
        res[r] = (same, nb, events, data, loss)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for r in range(2):
        same, nb, events, _, loss = res[r]
        assert same, r
        assert nb >= 3 and np.isfinite(loss)
        launches = [e for e in events if e[0] == "launch"]
        assert len(launches) == nb
        assert events[-1][0] == "finish"
    assert np.array_equal(res[0][3], res[1][3])      # replicas identical after the update
