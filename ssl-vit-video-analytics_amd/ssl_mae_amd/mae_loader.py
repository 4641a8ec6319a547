"""Clip loading and tube masking (reference: src/datasets/mae_loader.py).

LazyVideoMAEDataset (mae_loader.py:7-78) keeps the reference's constructor,
split-file parsing, sorted-*.jpg listing, frame-index rule (global numpy RNG),
black replacement frame for an unreadable file and zero clip for a missing or
empty directory.  What changes is where the per-pixel work runs:

  * transform=None (the MI355X path): __getitem__ returns the decoded uint8 frames
    [T,H,W,3] and a validity flag; `collate_frames` stacks a batch and
    `ClipNormalizer` ships it to HBM in ONE uint8 copy (1/4 of the fp32 bytes) and
    runs sm_frames_normalize, which applies the reference's transform
    (train_ssl_mae.py:137-141: /255, ImageNet mean/std) and its BGR channel swap
    (mae_loader.py:70-71) and lays the batch out as [B,3,T,H,W] fp32 — bit-identical
    to the reference's collated CPU clip;
  * transform=callable: the reference's behaviour verbatim (the callable runs per
    frame, then img[[2,1,0]] on tensors, stack, permute) — user code, on the host.

get_tube_mask (mae_loader.py:80-90) keeps the reference's signature and RNG stream:
the per-sample noise is drawn on the host from torch's global CPU generator exactly
as the reference draws it (B calls of torch.rand(L) == torch.rand(B, L)); the
ranking, the [B,T,L] expansion and the row-major compaction of masked token
indices run in one HIP kernel (sm_tube_mask).  The result is a bool tensor on the
GPU (the reference's `.to(device)` is then a no-op).  The kernel breaks ties in the
noise by lower index first, while the reference takes torch's CPU
`argsort(descending=True)`, which is not stable for L > 16.  The two can differ only
where equal noise values straddle the int(r*L) cut (~2e-5 per sample at L=784), and
the host removes exactly that case before the copy (`resolve_cut_ties`): one row sort
of the batch's noise in numpy (~0.5 ms at B=256, L=784) finds the samples whose
n_mask-th and (n_mask+1)-th largest values are equal, and for those samples only the
noise row is replaced by distinct values in the order of the reference's own
`torch.argsort(noise[b], descending=True)`.  The kernel's ranking then reproduces the
reference's selection by construction.
"""
import os

import numpy as np
import torch

from . import ops as K    # every kernel launch through the torch.ops.ssl_mae dispatcher

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


class LazyVideoMAEDataset(torch.utils.data.Dataset):
    """mae_loader.py:7-78 (see the module docstring for the transform=None path)."""

    def __init__(self, split_file, clip_len=32, stride=2, image_size=112, transform=None):
        self.clip_len = clip_len
        self.stride = stride
        self.image_size = image_size
        self.transform = transform
        self.samples = []
        if not os.path.exists(split_file):
            raise FileNotFoundError(f"Index file not found: {split_file}")
        with open(split_file, "r") as f:
            for line in f:
                parts = line.strip().split()
                if parts:
                    self.samples.append(parts[0])

    def __len__(self):
        return len(self.samples)

    def _load_frame(self, frame_path):
        from PIL import Image
        try:
            return Image.open(frame_path).convert("RGB")
        except Exception:
            return Image.new("RGB", (self.image_size, self.image_size), (0, 0, 0))

    def _indices(self, total):
        window = self.clip_len * self.stride
        if total < window:
            idx = np.linspace(0, total - 1, self.clip_len).astype(int)
        else:
            start = np.random.randint(0, total - window + 1)
            idx = np.arange(start, start + window, self.stride)
        return idx[:self.clip_len]

    def _empty(self):
        if self.transform is None:
            s = self.image_size
            return torch.zeros(self.clip_len, s, s, 3, dtype=torch.uint8), False
        return torch.zeros(3, self.clip_len, self.image_size, self.image_size)

    def __getitem__(self, index):
        video_dir = self.samples[index]
        if not os.path.exists(video_dir):
            return self._empty()
        names = sorted(f for f in os.listdir(video_dir) if f.endswith(".jpg"))
        if not names:
            return self._empty()
        imgs = [self._load_frame(os.path.join(video_dir, names[i])) for i in self._indices(len(names))]
        if self.transform is None:
            return torch.from_numpy(np.stack([np.asarray(im, dtype=np.uint8) for im in imgs])), True
        clip = []
        for img in imgs:
            img = self.transform(img)
            if isinstance(img, torch.Tensor):
                img = img[[2, 1, 0], :, :]
            clip.append(img)
        return torch.stack(clip).permute(1, 0, 2, 3)


def collate_frames(batch):
    """DataLoader collate for transform=None items: (uint8 [B,T,H,W,3], bool [B])."""
    frames = torch.stack([f for f, _ in batch])
    valid = torch.tensor([bool(v) for _, v in batch], dtype=torch.bool)
    return frames, valid


class ClipNormalizer:
    """Host frames -> normalised fp32 clip [B,3,T,H,W] in HBM (sm_frames_normalize)."""

    def __init__(self, mean=IMAGENET_MEAN, std=IMAGENET_STD, bgr_swap=True, device="cuda"):
        self.mean, self.std, self.bgr_swap, self.device = tuple(mean), tuple(std), bgr_swap, torch.device(device)

    def __call__(self, frames, valid=None):
        f = frames.to(self.device, non_blocking=True)
        v = None if valid is None else valid.to(self.device, non_blocking=True)
        return K.frames_normalize(f.contiguous(), self.mean, self.std, self.bgr_swap, v)


def resolve_cut_ties(noise, num_mask):
    """noise [B, L] fp32 (CPU): rows where equal values straddle the num_mask cut are
    replaced in place by distinct values ranked as the reference's
    torch.argsort(noise[b], descending=True) (mae_loader.py:86) ranks them; every other
    row is left untouched (the lower-index tie rule of sm_tube_mask cannot change
    which positions are selected there).  Returns the list of replaced rows."""
    B, L = noise.shape
    if num_mask <= 0 or num_mask >= L:
        return []
    s = np.sort(noise.numpy(), axis=1)
    rows = np.nonzero(s[:, L - num_mask] == s[:, L - num_mask - 1])[0].tolist()
    for b in rows:
        perm = torch.argsort(noise[b], descending=True)
        ranked = torch.empty(L, dtype=noise.dtype)
        ranked[perm] = torch.arange(L, 0, -1, dtype=noise.dtype)   # rank 0 -> largest
        noise[b] = ranked
    return rows


def tube_mask_from_noise(noise, num_frames, num_mask, device="cuda"):
    """noise [B, L] fp32 on the host -> (bool mask [B,T,L], int32 row-major index list) on
    `device`, selecting exactly the reference's argsort(descending)[:num_mask] per row."""
    noise = noise.clone()
    resolve_cut_ties(noise, num_mask)
    m8, idx = K.tube_mask(noise.to(device, non_blocking=True), num_frames, num_mask)
    return m8.view(torch.bool), idx


def tube_mask_with_index(batch_size, num_frames, num_patches, mask_ratio, device="cuda"):
    num_mask = int(mask_ratio * num_patches)
    noise = torch.rand(batch_size, num_patches)          # global CPU generator, reference order
    return tube_mask_from_noise(noise, num_frames, num_mask, device)


def get_tube_mask(batch_size, num_frames, num_patches, mask_ratio, device="cuda"):
    return tube_mask_with_index(batch_size, num_frames, num_patches, mask_ratio, device)[0]
