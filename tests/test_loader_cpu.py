"""Clip input pipeline on CPU.

The numpy oracle, fed by the host dataset's transform=None path (decoded uint8
frames, same index rule and RNG stream), reproduces the clips the reference's
LazyVideoMAEDataset returned (tests/golden/loader.npz) bit for bit, across all of
__getitem__'s branches (long/short video, missing/empty dir, corrupt frame)."""
import numpy as np
import pytest

import loader_fixture


def test_oracle_and_host_frames_match_reference(tmp_path):
    from oracle import loader_oracle as O
    from ssl_mae_amd.mae_loader import LazyVideoMAEDataset
    z, split, ref = loader_fixture.load(tmp_path)
    ds = LazyVideoMAEDataset(split, clip_len=int(z["clip_len"]), stride=int(z["stride"]),
                             image_size=int(z["size"]), transform=None)
    assert len(ds) == len(ref)
    np.random.seed(int(z["seed"]))
    items = [ds[i] for i in range(len(ds))]
    for i, ((frames, valid), r) in enumerate(zip(items, ref)):
        got = O.normalize_clip(frames.numpy(), z["mean"], z["std"]) if valid else np.zeros_like(r)
        assert got.dtype == r.dtype and got.shape == r.shape, i
        assert np.array_equal(got, r), i
    assert [bool(v) for _, v in items] == [True, True, False, False, True, True]


def test_host_transform_path_is_reference_behaviour(tmp_path):
    """transform=callable keeps the reference's per-frame path (user code on the host)."""
    import torch
    from ssl_mae_amd.mae_loader import LazyVideoMAEDataset
    z, split, ref = loader_fixture.load(tmp_path)
    mean = torch.as_tensor(z["mean"])[:, None, None]
    std = torch.as_tensor(z["std"])[:, None, None]

    def tf(img):
        x = torch.from_numpy(np.asarray(img, dtype=np.uint8).copy()).permute(2, 0, 1).to(torch.float32) / 255
        return (x - mean) / std
    ds = LazyVideoMAEDataset(split, clip_len=int(z["clip_len"]), stride=int(z["stride"]),
                             image_size=int(z["size"]), transform=tf)
    np.random.seed(int(z["seed"]))
    for i, r in enumerate(ref):
        assert np.array_equal(ds[i].numpy(), r), i


def test_missing_split_file_raises(tmp_path):
    from ssl_mae_amd.mae_loader import LazyVideoMAEDataset
    with pytest.raises(FileNotFoundError):
        LazyVideoMAEDataset(str(tmp_path / "nope.txt"))


def test_frame_index_rule():
    from oracle import loader_oracle as O
    np.random.seed(0)
    assert list(O.frame_indices(3, 8, 2)) == [0, 0, 0, 0, 1, 1, 1, 2]      # short: linspace
    for total in (16, 17, 40):
        idx = O.frame_indices(total, 8, 2)
        assert len(idx) == 8 and np.all(np.diff(idx) == 2) and idx[-1] < total
