"""CPU ORACLE — TEST INFRASTRUCTURE ONLY.

numpy restatement of the reference's clip loading (src/datasets/mae_loader.py:7-78)
with the transform of src/train_ssl_mae.py:137-141.  Only `tests/` imports it, as
the checker; the product path (ssl_mae_amd.mae_loader + sm_frames_normalize) never
does.  Pinned by tests/golden/loader.npz (make_golden_loader.py runs the reference
dataset; tests/test_loader_cpu.py checks this module against it).

  frame_indices   mae_loader.py:46-59  (global numpy RNG: np.random.randint for
                                        the start of a long video, linspace for a
                                        short one, truncated to clip_len)
  list_frames     mae_loader.py:39     (sorted *.jpg names)
  normalize_clip  train_ssl_mae.py:137-141 + mae_loader.py:70-77:
                  (u8 / 255 - mean) / std in fp32, channels reversed, [C,T,H,W]
  zero clip       mae_loader.py:35-43  (missing directory or no frames)
"""
import os

import numpy as np


def list_frames(video_dir):
    return sorted(f for f in os.listdir(video_dir) if f.endswith(".jpg"))


def frame_indices(total_frames, clip_len, stride):
    window = clip_len * stride
    if total_frames < window:
        idx = np.linspace(0, total_frames - 1, clip_len).astype(int)
    else:
        start = np.random.randint(0, total_frames - window + 1)
        idx = np.arange(start, start + window, stride)
    return idx[:clip_len]


def normalize_clip(frames_u8, mean, std):
    """frames [T,H,W,3] uint8 RGB -> [3,T,H,W] fp32, BGR order."""
    x = frames_u8.astype(np.float32) / np.float32(255)
    x = (x - np.asarray(mean, np.float32)) / np.asarray(std, np.float32)
    return np.ascontiguousarray(x[..., ::-1].transpose(3, 0, 1, 2))
