"""Portable deterministic parameter rule shared by the golden-fixture generator,
the CPU oracle and the HIP model.

The reference initialises with torch RNG (xavier / trunc_normal / kaiming;
`src/models/mae_vit_adapter.py:57-73`, `src/models/tiny_vit.py:17-18`).  Parity
needs the SAME numbers on both sides without shipping 120 MB of weights, so every
tensor is drawn from numpy's PCG64 seeded by crc32(parameter name):

* weights with ndim >= 2: N(0, 1) / sqrt(fan_in)           (fan_in = prod(shape[1:]))
* norm / BN affine weights (1-D, name ends with 'weight'): 1 + 0.1 N(0, 1)
* biases, position embeddings, mask token: 0.02 N(0, 1)
* BN running_mean 0, running_var 1, num_batches_tracked 0 (torch defaults)
"""
import zlib

import numpy as np
import torch


def param_value(name: str, shape) -> np.ndarray:
    rng = np.random.default_rng(zlib.crc32(name.encode()))
    shape = tuple(int(s) for s in shape)
    z = rng.standard_normal(shape)
    if len(shape) >= 2 and not name.endswith(("pos_embed", "mask_token")):
        fan_in = int(np.prod(shape[1:]))
        v = z / np.sqrt(fan_in)
    elif name.endswith("weight"):
        v = 1.0 + 0.1 * z
    else:
        v = 0.02 * z
    return v.astype(np.float32)


@torch.no_grad()
def apply_rule(module: torch.nn.Module) -> None:
    """Overwrite every parameter of `module` (names relative to it) in place."""
    for name, p in module.named_parameters():
        p.copy_(torch.from_numpy(param_value(name, p.shape)).to(p.device, p.dtype))
    for name, b in module.named_buffers():
        if name.endswith("running_mean"):
            b.zero_()
        elif name.endswith("running_var"):
            b.fill_(1.0)
        elif name.endswith("num_batches_tracked"):
            b.zero_()


IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def synthetic_clip(B: int, T: int, S: int, seed: int = 1234) -> np.ndarray:
    """fp32 [B,3,T,S,S] = (U[0,1) - mean_c) / std_c, numpy PCG64 seeded."""
    rng = np.random.default_rng(seed)
    u = rng.random((B, 3, T, S, S), dtype=np.float32)
    mean = np.asarray(IMAGENET_MEAN, np.float32).reshape(1, 3, 1, 1, 1)
    std = np.asarray(IMAGENET_STD, np.float32).reshape(1, 3, 1, 1, 1)
    return ((u - mean) / std).astype(np.float32)
