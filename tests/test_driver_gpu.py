"""The reference's driver on the GPU: `main()` end to end on a small synthetic
frame dataset (split file + jpg frame directories, as `LazyVideoMAEDataset`
reads them, mae_loader.py:7-78), the reference's encoder-only checkpoint file,
and a full-state resume that continues bit-for-bit (train_ssl_mae.py:129-194)."""
import os

import numpy as np
import pytest
import torch
import yaml

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _dataset(root, n_videos=3, n_frames=10, size=64):
    from PIL import Image
    rng = np.random.default_rng(0)
    lines = []
    for v in range(n_videos):
        d = root / f"video_{v}"
        d.mkdir()
        for f in range(n_frames if v else 3):        # video_0 is short: linspace branch
            Image.fromarray(rng.integers(0, 256, (size, size, 3), dtype=np.uint8)).save(d / f"{f:05d}.jpg")
        lines.append(f"{d} {v}")
    lines.append(f"{root / 'missing_video'} 9")       # zero clip branch
    split = root / "split.txt"
    split.write_text("\n".join(lines) + "\n")
    return split


def _config(root, split, epochs):
    cfg = {"dataset": {"train_split": str(split), "clip_len": 4, "stride": 2, "image_size": 64},
           "model": {"type": "tiny_vit_21m_variant", "decoder_embed_dim": 384, "decoder_depth": 2,
                     "decoder_num_heads": 6},
           "ssl": {"mask_ratio": 0.75, "mask_strategy": "tube", "norm_pix_loss": True},
           "training": {"epochs": epochs, "batch_size": 2, "num_workers": 0, "lr": 5e-4, "weight_decay": 0.05,
                        "save_dir": str(root / "results" / "tinymae_test"), "log_interval": 20}}
    p = root / f"cfg_{epochs}.yaml"
    p.write_text(yaml.safe_dump(cfg))
    return p


def test_main_runs_saves_and_resumes_bit_exact(tmp_path, monkeypatch):
    from ssl_mae_amd import train_ssl_mae as TR
    monkeypatch.chdir(tmp_path)
    split = _dataset(tmp_path)
    cfg12 = _config(tmp_path, split, 12)
    a = TR.main(["--config", str(cfg12), "--max-steps", "1"])
    save_dir = tmp_path / "results" / "tinymae_test"
    enc = torch.load(save_dir / "encoder_ep10.pth", map_location="cpu", weights_only=True)
    assert set(enc) == set(a.encoder.state_dict())             # the reference's encoder-only file
    assert (save_dir / "last_state.pth").exists()
    pa = {k: v.detach().cpu().clone() for k, v in a.state_dict().items()}
    assert all(torch.isfinite(v).all() for v in pa.values() if v.is_floating_point())
    # resume from the epoch-10 state and finish epochs 11-12: identical parameters,
    # optimizer moments and BN running statistics
    b = TR.main(["--config", str(cfg12), "--max-steps", "1", "--resume", str(save_dir / "last_state.pth")])
    pb = {k: v.detach().cpu() for k, v in b.state_dict().items()}
    for k in pa:
        assert torch.equal(pa[k], pb[k]), k


def test_rng_state_round_trip_device_stream():
    """The device generator's state (seed AND offset) is saved, so torch device RNG
    use after a resume continues the stream instead of repeating it from the start."""
    import torch
    from ssl_mae_amd.checkpoint import _rng_state, _set_rng_state
    torch.cuda.manual_seed_all(11)
    torch.rand(1000, device="cuda")
    st = _rng_state()
    a = torch.rand(16, device="cuda").cpu()
    torch.rand(5000, device="cuda")
    _set_rng_state(st)
    b = torch.rand(16, device="cuda").cpu()
    assert torch.equal(a, b)
