"""The benchmarked memory policy has its own test: a B = 256 step under
the device-memory arena with the policy bench.py's auto rule picks there (stages 0-2 resident),
in a child process exactly as bench.py sets it up (tests/policy_child.py), checked against

* the reference's loss formula (/root/reference/src/train_ssl_mae.py:26-31,72-84: patchify,
  unbiased norm_pix, masked MSE) evaluated in fp32 torch on the step's own pred and mask, to 1e-4;
* the BatchNorm counters the reference's checkpointed forward + recompute leaves
  (train_ssl_mae.py:66-91 with tiny_vit.py:170-175: stem once, stages 0-2 twice per step);
* bit-identity with the same step under the other policy (stages 1-2 resident, stage 0
  lite-resident) on the same clips, mask and dropout seeds: loss, flat gradients, parameters
  after AdamW and every BN running buffer.
Every request must have been served from the arena's heap."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.gpu_fresh
@pytest.mark.timeout(600)
def test_bench_policy_b256_under_arena():
    import gc
    free = None
    try:
        import torch
        if torch.cuda.is_initialized():
            gc.collect()
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
            free = torch.cuda.mem_get_info()[0] / 2 ** 30
    except Exception:
        pass
    r = subprocess.run([sys.executable, os.path.join(HERE, "policy_child.py")], capture_output=True, text=True,
                       timeout=540)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    # what bench.py runs at B = 256 under the arena (a fresh process: the whole HBM to size the arena)
    assert d["auto"] == [[0, 1, 2], []], (d["auto"], d["arena"].get("capacity", 0) / 2 ** 30, free)
    a, b = d["runs"]
    assert a["resident"] == [0, 1, 2] and b["resident"] == [1, 2] and b["lite"] == [0]
    for run in (a, b):
        assert run["grad_finite"]
        assert abs(run["loss"] - run["ref_loss"]) < 1e-4 * abs(run["ref_loss"]), run
        assert run["mask_rows"] == 256 * 8 * 588
        for name, v in run["counters"].items():
            if ".stages.3." in name:
                continue
            assert v == (1 if "patch_embed" in name else 2), (name, v)
    assert a["loss"] == b["loss"]
    assert a["grads"] == b["grads"] and a["params"] == b["params"] and a["buffers"] == b["buffers"]
    assert a["peak_gib"] > b["peak_gib"]                      # resident stage 0 keeps more in HBM
    st = d["arena"]
    assert st["hipmalloc_requests"] == 0 and st["outside_bytes"] == 0
