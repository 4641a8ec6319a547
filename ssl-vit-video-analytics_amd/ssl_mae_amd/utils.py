"""Support API of the reference (src/utils.py:10-26, 73-77)."""
import random
from pathlib import Path

import numpy as np
import torch
import yaml


def load_config(path):
    path = Path(path)
    if not path.exists():
        raise RuntimeError(f"[ERROR] Config not found: {path}")
    with open(path, "r", encoding="utf-8") as f:
        cfg = yaml.safe_load(f)
    return cfg or {}


def set_seed(seed):
    seed = int(seed)
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)


def save_checkpoint(state, filename):
    filename = Path(filename)
    filename.parent.mkdir(parents=True, exist_ok=True)
    torch.save(state, filename)
