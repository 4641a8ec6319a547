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
