"""Tube-mask tie handling on the host (reference
src/datasets/mae_loader.py:80-90).

sm_tube_mask ranks noise by value, ties by lower index.  The reference selects
torch.argsort(noise, descending=True)[:num_mask], whose CPU sort is not stable, so
the two can disagree exactly when equal values straddle the num_mask cut.
`resolve_cut_ties` rewrites those rows (only those) before the copy.  These tests
construct such ties and check, with a CPU restatement of the kernel's rank rule,
that the selection equals the reference's argsort selection; the GPU half is
tests/test_kernels_gpu.py::test_tube_mask_constructed_cut_ties."""
import numpy as np
import torch


def kernel_rule_select(noise, num_mask):
    """CPU restatement of tube_mask_kernel's ranking (csrc/mae.hip): rank(i) = #{j:
    v_j > v_i} + #{j < i: v_j == v_i}; masked iff rank < num_mask."""
    v = noise.numpy()
    L = v.shape[0]
    gt = (v[None, :] > v[:, None]).sum(1)
    eq_lower = np.array([(v[:i] == v[i]).sum() for i in range(L)])
    return (gt + eq_lower) < num_mask


def reference_select(noise, num_mask):
    """mae_loader.py:86: torch.argsort(noise, descending=True)[:num_mask]."""
    sel = np.zeros(noise.shape[0], dtype=bool)
    sel[torch.argsort(noise, descending=True)[:num_mask].numpy()] = True
    return sel


def constructed_cut_ties(B, L, num_mask, seed):
    """Noise rows where several values equal to the one at rank num_mask - 1 sit on
    both sides of the cut (drawn as torch.rand draws, then tied)."""
    g = torch.Generator().manual_seed(seed)
    noise = torch.rand(B, L, generator=g)
    for b in range(B):
        order = torch.argsort(noise[b], descending=True)
        v = noise[b, order[num_mask - 1]].item()
        # ranks num_mask-3 .. num_mask+2 all take the value at the cut: 6-way tie, 3 in / 3 out
        noise[b, order[num_mask - 3:num_mask + 3]] = v
    return noise


def test_constructed_ties_differ_without_resolution():
    """The constructed ties are real cases: the lower-index rule alone would disagree
    with the reference on some rows (otherwise the test below proves nothing)."""
    from ssl_mae_amd.mae_loader import resolve_cut_ties  # noqa: F401
    L, nm = 784, 588
    noise = constructed_cut_ties(32, L, nm, seed=11)
    differ = sum(not np.array_equal(kernel_rule_select(noise[b], nm), reference_select(noise[b], nm))
                 for b in range(32))
    assert differ > 0


def test_resolved_rows_select_as_reference():
    from ssl_mae_amd.mae_loader import resolve_cut_ties
    for L, nm, seed in ((784, 588, 11), (196, 176, 12), (784, 392, 13), (64, 48, 14)):
        orig = constructed_cut_ties(16, L, nm, seed)
        noise = orig.clone()
        rows = resolve_cut_ties(noise, nm)
        assert rows == list(range(16))
        for b in range(16):
            assert np.array_equal(kernel_rule_select(noise[b], nm), reference_select(orig[b], nm)), (L, nm, b)
            assert len(set(noise[b].tolist())) == L   # distinct: the rank rule has no ties left


def test_rows_without_cut_ties_untouched():
    from ssl_mae_amd.mae_loader import resolve_cut_ties
    torch.manual_seed(5)
    noise = torch.rand(256, 784)
    noise[3, :10] = noise[3, 10]              # a tie far from the cut (not straddling)
    orig = noise.clone()
    tied = constructed_cut_ties(1, 784, 588, seed=21)
    noise[7] = tied[0]
    orig[7] = tied[0]
    rows = resolve_cut_ties(noise, 588)
    assert rows == [7]
    keep = [b for b in range(256) if b != 7]
    assert torch.equal(noise[keep], orig[keep])
    for b in (3, 7, 100):
        assert np.array_equal(kernel_rule_select(noise[b], 588), reference_select(orig[b], 588))


def test_no_cut_for_ratio_zero_or_one():
    from ssl_mae_amd.mae_loader import resolve_cut_ties
    noise = torch.zeros(4, 16)
    assert resolve_cut_ties(noise.clone(), 0) == [] and resolve_cut_ties(noise.clone(), 16) == []
    assert resolve_cut_ties(noise, 8) == [0, 1, 2, 3]   # all equal: every row straddles
    for b in range(4):
        assert np.array_equal(kernel_rule_select(noise[b], 8), reference_select(torch.zeros(16), 8))
