"""sm_frames_normalize through the C ABI: the reference's collated clip bit for bit
(tests/golden/loader.npz), plus the BASELINE frame size against the oracle."""
import numpy as np
import pytest
import torch

import loader_fixture

pytestmark = pytest.mark.gpu


def test_normalizer_matches_reference_clips(tmp_path):
    from ssl_mae_amd.mae_loader import ClipNormalizer, LazyVideoMAEDataset, collate_frames
    z, split, ref = loader_fixture.load(tmp_path)
    ds = LazyVideoMAEDataset(split, clip_len=int(z["clip_len"]), stride=int(z["stride"]),
                             image_size=int(z["size"]), transform=None)
    np.random.seed(int(z["seed"]))
    frames, valid = collate_frames([ds[i] for i in range(len(ds))])
    clip = ClipNormalizer(mean=z["mean"], std=z["std"])(frames, valid)
    assert clip.shape == (len(ref), 3, int(z["clip_len"]), int(z["size"]), int(z["size"]))
    assert np.array_equal(clip.cpu().numpy(), np.stack(ref))


@pytest.mark.parametrize("B,T,H,W,offset", [(4, 8, 224, 224, 0), (2, 3, 7, 9, 0), (1, 2, 8, 8, 1)])
def test_normalizer_vs_oracle(B, T, H, W, offset):
    from oracle import loader_oracle as O
    from ssl_mae_amd import kernels as K
    rng = np.random.default_rng(B * T + H)
    u8 = rng.integers(0, 256, (B, T, H, W, 3), dtype=np.uint8)
    if offset:   # frames start 1 byte into the allocation: scalar path
        buf = torch.empty(u8.size + 1, dtype=torch.uint8, device="cuda")
        buf[1:].copy_(torch.from_numpy(u8.reshape(-1)))
        f = buf[1:].view(B, T, H, W, 3)
    else:
        f = torch.from_numpy(u8).cuda()
    valid = torch.tensor([i != 1 for i in range(B)], device="cuda")
    out = K.frames_normalize(f, (0.485, 0.456, 0.406), (0.229, 0.224, 0.225), True, valid).cpu().numpy()
    for b in range(B):
        exp = O.normalize_clip(u8[b], (0.485, 0.456, 0.406), (0.229, 0.224, 0.225)) if b != 1 else 0
        assert np.array_equal(out[b], np.broadcast_to(exp, out[b].shape)), b
