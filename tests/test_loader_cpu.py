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


def test_finetune_checkpoint_bridge(tmp_path):
    """load_pretrained_ssl (train_finetune.py:43-63) reads both the MAE driver's
    encoder-only file (no prefix, train_ssl_mae.py:190-194) and an `encoder.`-prefixed
    full state; the reference's loader silently skips the former."""
    import torch
    from ssl_mae_amd.finetune import VideoClassifier, load_pretrained_ssl
    from ssl_mae_amd.mae_vit_adapter import TinyVideoMAE
    from ssl_mae_amd.tiny_vit import tiny_vit_21m_variant
    cfg = {"dataset": {"clip_len": 4, "image_size": 112},
           "model": {"decoder_embed_dim": 384, "decoder_depth": 1, "decoder_num_heads": 6}}
    torch.manual_seed(0)
    mae = TinyVideoMAE(tiny_vit_21m_variant(img_size=112), cfg)
    enc = mae.encoder.state_dict()
    torch.save(enc, tmp_path / "encoder_ep10.pth")
    torch.save({"model": mae.state_dict()}, tmp_path / "full.pth")
    for f in ("encoder_ep10.pth", "full.pth"):
        torch.manual_seed(1)
        clf = VideoClassifier(101)
        assert load_pretrained_ssl(clf, str(tmp_path / f))
        got = clf.backbone.state_dict()
        assert set(got) == set(enc)
        for k, v in enc.items():
            assert torch.equal(got[k], v), (f, k)
    assert not load_pretrained_ssl(VideoClassifier(5), str(tmp_path / "missing.pth"))
