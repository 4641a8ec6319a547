"""Rebuild the frame tree of tests/golden/loader.npz under a temp directory."""
import os

import numpy as np

from conftest import GOLDEN


def load(tmp_path):
    z = np.load(os.path.join(GOLDEN, "loader.npz"))
    for i, name in enumerate(z["names"]):
        p = os.path.join(str(tmp_path), str(name))
        os.makedirs(os.path.dirname(p), exist_ok=True)
        with open(p, "wb") as f:
            f.write(z[f"file{i}"].tobytes())
    os.makedirs(os.path.join(str(tmp_path), "empty"), exist_ok=True)
    split = os.path.join(str(tmp_path), "split.txt")
    with open(split, "w") as f:
        for d in z["dirs"]:
            f.write(f"{os.path.join(str(tmp_path), str(d))} 3\n")
        f.write("\n")
    clips = [z[f"clip{i}"] for i in range(len(z["dirs"]))]
    return z, split, clips
