"""The device-memory arena under the real step: two bf16 MAE steps (stage 0
resident) with the overlapped RCCL all-reduce on its side stream give the same
losses and parameters under the arena as under PyTorch's caching allocator, and
every request was served from the arena's heap (none fell back to hipMalloc)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _run(mode):
    try:   # this process's cached blocks back to the device before the child takes its heap
        import torch
        if torch.cuda.is_initialized():
            torch.cuda.empty_cache()
    except Exception:
        pass
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    r = subprocess.run([sys.executable, os.path.join(HERE, "arena_child.py"), mode, str(port)],
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.timeout(600)
def test_arena_step_matches_caching_allocator():
    a = _run("arena")
    c = _run("caching")
    st = a["arena"]
    assert st["capacity"] > 16 * 2 ** 30 and st["requests"] > 100
    assert st["hipmalloc_requests"] == 0 and st["outside_bytes"] == 0
    assert 0 < st["peak"] <= st["capacity"]
    assert a["launched"] == c["launched"] == 0                 # every bucket reduced and the hook reset
    for la, lc in zip(a["losses"], c["losses"]):
        assert abs(la - lc) <= 1e-6 * abs(lc), (a["losses"], c["losses"])
    for n, v in c["param_sums"].items():
        assert abs(a["param_sums"][n] - v) <= 1e-6 * max(1.0, abs(v)), n
