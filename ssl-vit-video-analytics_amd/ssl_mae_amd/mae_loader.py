"""Tube masking (reference: src/datasets/mae_loader.py:80-90).

`get_tube_mask(batch_size, num_frames, num_patches, mask_ratio)` keeps the
reference's signature and RNG stream: the per-sample noise is drawn on the host
from torch's global CPU generator exactly as the reference draws it (B calls of
torch.rand(L) == torch.rand(B, L)); the ranking, the [B,T,L] expansion and the
row-major compaction of masked token indices run in one HIP kernel
(sm_tube_mask).  The result is a bool tensor on the GPU (the reference's
`.to(device)` is then a no-op).  Ties in the noise are broken by lower index
first; the reference's torch CPU argsort is not stable for L > 16, so a tie that
straddles the int(r*L) cut (probability ~2e-5 per sample at L=784) may resolve
differently — see DESIGN.md.
"""
import torch

from . import kernels as K


def tube_mask_with_index(batch_size, num_frames, num_patches, mask_ratio, device="cuda"):
    num_mask = int(mask_ratio * num_patches)
    noise = torch.rand(batch_size, num_patches)          # global CPU generator, reference order
    noise = noise.to(device, non_blocking=True)
    m8, idx = K.tube_mask(noise, num_frames, num_mask)
    return m8.view(torch.bool), idx


def get_tube_mask(batch_size, num_frames, num_patches, mask_ratio, device="cuda"):
    return tube_mask_with_index(batch_size, num_frames, num_patches, mask_ratio, device)[0]
