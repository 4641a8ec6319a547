"""Generate tests/golden/loader.npz by RUNNING the reference's LazyVideoMAEDataset.

Build container only (the reference never travels).  Loads
src/datasets/mae_loader.py by file path (HF `datasets` shadows src/datasets) and
runs it over a small synthetic frame tree covering every branch of
`__getitem__` (mae_loader.py:33-78): a long video (random start, stride
window), a short one (linspace indices), a missing directory, an empty
directory, and a video with a corrupt .jpg (black replacement frame) plus a
non-.jpg file that must be ignored.

torchvision is not installed here.  The reference's transform
(train_ssl_mae.py:137-141: PILToTensor, ConvertImageDtype(float), Normalize) is
supplied as torch CPU ops following torchvision's published algorithm:
HWC uint8 -> CHW, `.to(float32) / 255`, then `(x - mean[:,None,None]) /
std[:,None,None]` with fp32 mean/std tensors.  Parity of that transform is thus
pinned to torchvision's documented arithmetic, the loader logic to the reference.

Output (data only): the JPEG bytes of every file, the split lines, the numpy
seed and the clips the reference returned.

    python tests/golden/make_golden_loader.py
"""
import importlib.util
import io
import os
import sys
import tempfile

import numpy as np
import torch
from PIL import Image

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/src/datasets/mae_loader.py"
MEAN = [0.485, 0.456, 0.406]
STD = [0.229, 0.224, 0.225]
SIZE, CLIP_LEN, STRIDE, SEED = 32, 4, 2, 1234


def transform(img):
    x = torch.from_numpy(np.asarray(img, dtype=np.uint8).copy()).permute(2, 0, 1).contiguous()
    x = x.to(torch.float32) / 255
    m = torch.as_tensor(MEAN, dtype=torch.float32)[:, None, None]
    s = torch.as_tensor(STD, dtype=torch.float32)[:, None, None]
    return (x - m) / s


def make_tree(root):
    rng = np.random.default_rng(5)
    files = {}

    def jpg(rel, arr):
        b = io.BytesIO()
        Image.fromarray(arr).save(b, format="JPEG", quality=90)
        files[rel] = b.getvalue()

    for i in range(20):
        jpg(f"long/{i:05d}.jpg", rng.integers(0, 256, (SIZE, SIZE, 3), dtype=np.uint8))
    for i in range(3):
        jpg(f"short/img_{i}.jpg", rng.integers(0, 256, (SIZE, SIZE, 3), dtype=np.uint8))
    for i in range(9):
        jpg(f"corrupt/{i:03d}.jpg", rng.integers(0, 256, (SIZE, SIZE, 3), dtype=np.uint8))
    files["corrupt/004.jpg"] = b"not a jpeg"
    files["corrupt/notes.txt"] = b"ignored"
    for rel, data in files.items():
        p = os.path.join(root, rel)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        with open(p, "wb") as f:
            f.write(data)
    os.makedirs(os.path.join(root, "empty"), exist_ok=True)
    return files


def main():
    spec = importlib.util.spec_from_file_location("ref_mae_loader", REF)
    ref = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ref)
    with tempfile.TemporaryDirectory() as root:
        files = make_tree(root)
        dirs = ["long", "short", "missing", "empty", "corrupt", "long"]
        split = os.path.join(root, "split.txt")
        with open(split, "w") as f:
            for d in dirs:
                f.write(f"{os.path.join(root, d)} 3\n")
            f.write("\n")                                  # blank line: skipped
        ds = ref.LazyVideoMAEDataset(split, clip_len=CLIP_LEN, stride=STRIDE, image_size=SIZE, transform=transform)
        np.random.seed(SEED)
        clips = [ds[i].numpy() for i in range(len(ds))]
    out = {"dirs": np.array(dirs), "names": np.array(sorted(files)), "seed": np.int64(SEED),
           "size": np.int64(SIZE), "clip_len": np.int64(CLIP_LEN), "stride": np.int64(STRIDE),
           "mean": np.array(MEAN, np.float32), "std": np.array(STD, np.float32)}
    for i, name in enumerate(sorted(files)):
        out[f"file{i}"] = np.frombuffer(files[name], dtype=np.uint8)
    for i, c in enumerate(clips):
        out[f"clip{i}"] = c
    np.savez_compressed(os.path.join(HERE, "loader.npz"), **out)
    print("wrote loader.npz:", len(clips), "clips", [c.shape for c in clips])


if __name__ == "__main__":
    main()
