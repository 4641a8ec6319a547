"""Device-memory arena (csrc/arena.cpp): placement and coalescing, checked over a
host buffer attached to an unused device slot (sm_arena_attach; no HIP call is
made and arena memory is never dereferenced)."""
import ctypes
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "ssl-vit-video-analytics_amd"))

from ssl_mae_amd import arena  # noqa: E402

MIB = 1 << 20


def _attach(slot, cap):
    lib = arena.library()
    base = 1 << 40                              # a fake range: the arena never dereferences its memory
    assert lib.sm_arena_attach(slot, ctypes.c_void_p(base), cap) == 0
    assert lib.sm_arena_attach(slot, ctypes.c_void_p(base), cap) == -1   # slot taken
    return lib, base


def test_exports():
    lib = arena.library()
    for sym in ("sm_arena_alloc", "sm_arena_free", "sm_arena_stats", "sm_arena_reset_peak", "sm_arena_attach"):
        assert hasattr(lib, sym)


def test_best_fit_and_coalescing():
    slot = 13
    lib, base = _attach(slot, 64 * MIB)
    a = lib.sm_arena_alloc(1 * MIB, slot, None)
    b = lib.sm_arena_alloc(4 * MIB, slot, None)
    c = lib.sm_arena_alloc(1 * MIB, slot, None)
    d = lib.sm_arena_alloc(2 * MIB, slot, None)
    assert [a, b, c, d] == [base, base + MIB, base + 5 * MIB, base + 6 * MIB]
    lib.sm_arena_free(b, 4 * MIB, slot, None)
    # best fit: the 4 MiB hole beats the 56 MiB tail, lowest address first
    e = lib.sm_arena_alloc(3 * MIB, slot, None)
    assert e == b
    f = lib.sm_arena_alloc(1 * MIB, slot, None)
    assert f == b + 3 * MIB
    s = arena.stats(slot)
    assert s["in_use"] == 8 * MIB and s["peak"] == 8 * MIB and s["free_blocks"] == 1
    for p, n in ((a, MIB), (c, MIB), (e, 3 * MIB), (d, 2 * MIB), (f, MIB)):
        lib.sm_arena_free(p, n, slot, None)
    s = arena.stats(slot)
    assert s["in_use"] == 0 and s["free_blocks"] == 1 and s["largest_free"] == 64 * MIB
    lib.sm_arena_reset_peak(slot)
    assert arena.stats(slot)["peak"] == 0


def test_random_sequence_no_overlap_full_coalesce():
    slot = 14
    cap = 256 * MIB
    lib, base = _attach(slot, cap)
    rng = np.random.default_rng(5)
    live = {}
    for step in range(4000):
        if live and (rng.random() < 0.45 or len(live) > 60):
            p = list(live)[rng.integers(len(live))]
            lib.sm_arena_free(p, live.pop(p), slot, None)
            continue
        n = int(rng.choice([1, 700, 4096, 100_000, MIB, 3 * MIB + 17, 9 * MIB]))
        p = lib.sm_arena_alloc(n, slot, None)
        if p is None:                 # full: the hipMalloc fallback fails without a GPU
            continue
        assert p % 512 == 0 and base <= p and p + n <= base + cap
        live[p] = n
        if step % 97 == 0:
            spans = sorted((q, q + ((m + 511) // 512) * 512) for q, m in live.items())
            assert all(e0 <= s1 for (_, e0), (s1, _) in zip(spans, spans[1:])), "overlapping blocks"
            assert arena.stats(slot)["in_use"] == sum(e - s for s, e in spans)
    for p, n in live.items():
        lib.sm_arena_free(p, n, slot, None)
    s = arena.stats(slot)
    assert s["in_use"] == 0 and s["free_blocks"] == 1 and s["largest_free"] == cap


def test_zero_size_request_gets_a_block():
    slot = 15
    lib, base = _attach(slot, 4 * MIB)
    p = lib.sm_arena_alloc(0, slot, None)
    assert p == base
    lib.sm_arena_free(p, 0, slot, None)
    assert arena.stats(slot)["in_use"] == 0


@pytest.mark.parametrize("policy_cap, expect", [(0.0, (1, 2)), (200.0, (1, 2)), (281.0, (0, 1, 2))])
def test_stage0_resident_policy_needs_arena(monkeypatch, policy_cap, expect):
    """auto_resident_stages: stage 0 resident only under an arena whose capacity
    holds the predicted 263 GiB at B = 256 (T = 8, 224^2, bf16)."""
    import torch
    from ssl_mae_amd import tiny_vit as TV

    class Props:
        total_memory = 288 * 2 ** 30
    monkeypatch.setattr(torch.cuda, "get_device_properties", lambda d: Props())
    monkeypatch.setattr(arena, "active", lambda: policy_cap > 0)
    monkeypatch.setattr(arena, "capacity_gib", lambda d=None: policy_cap)
    assert TV.auto_resident_stages(256 * 8, 224, True, "cuda") == expect
    assert TV.auto_lite_stages(256 * 8, 224, True, "cuda", expect) == ((0,) if expect == (1, 2) else ())


@pytest.mark.parametrize("cap, expect", [(0.0, ()), (281.0, (0,))])
def test_small_stage0_resident_needs_arena(monkeypatch, cap, expect):
    """C3 ViT-Small (depths 2,2,12,2 + 8-layer decoder): stage 0 resident (231.2 GiB at B = 256)
    only under the arena; its other resident policies do not fit 288 GB."""
    import torch
    from ssl_mae_amd import tiny_vit as TV

    class Props:
        total_memory = 288 * 2 ** 30
    monkeypatch.setattr(torch.cuda, "get_device_properties", lambda d: Props())
    monkeypatch.setattr(arena, "active", lambda: cap > 0)
    monkeypatch.setattr(arena, "capacity_gib", lambda d=None: cap)
    assert TV.auto_resident_stages(256 * 8, 224, True, "cuda", key=((2, 2, 12, 2), 8)) == expect
    assert TV.auto_lite_stages(256 * 8, 224, True, "cuda", expect, key=((2, 2, 12, 2), 8)) == ()


def test_explicit_policy_checked_against_arena_capacity(monkeypatch):
    """An explicit resident / lite request whose predicted peak exceeds the arena's capacity
    raises a RuntimeError naming both sizes before the step (instead of the arena meeting the
    failing request inside the step, csrc/arena.cpp); the capacity is read from a host-attached
    arena slot.  C3 ViT-Small with stage 2 resident was measured out of memory at > 300 GB."""
    from ssl_mae_amd import tiny_vit as TV
    slot = 12
    _attach(slot, int(281.4 * 2 ** 30))
    monkeypatch.setattr(arena, "active", lambda: True)
    small, tiny = ((2, 2, 12, 2), 8), ((2, 2, 6, 2), 4)
    F, S = 256 * 8, 224
    with pytest.raises(RuntimeError, match=r"needs 279\.4 GiB") as ei:
        TV.check_memory_policy(F, S, True, slot, (2,), (), key=small)
    msg = str(ei.value)
    assert "lower bound" in msg and "281.4 GiB" in msg and "arena" in msg
    with pytest.raises(RuntimeError, match="lower bound"):          # a superset of an OOM policy
        TV.check_memory_policy(F, S, True, slot, (1, 2), (), key=small)
    TV.check_memory_policy(F, S, True, slot, (0,), (), key=small)    # 231.2 GiB measured: fits
    TV.check_memory_policy(F, S, True, slot, (0, 1, 2), (), key=tiny)   # 263.1 GiB: fits
    TV.check_memory_policy(F, S, True, slot, (1, 2), (0,), key=tiny)    # 229.8 GiB: fits
    TV.check_memory_policy(64, S, True, slot, (2,), (), key=small)   # small batches always fit
    with pytest.raises(RuntimeError, match="measured"):               # fp32 doubles the activations
        TV.check_memory_policy(F, S, False, slot, (0, 1, 2), (), key=tiny)
    pred, basis = TV.predicted_peak_gib(F, S, True, (1,), (), key=small)
    assert basis == "estimate" and 184.0 < pred < 288.0
    assert TV.predicted_peak_gib(F, S, True, (0,), key=((9, 9, 9, 9), 1)) == (None, None)


def test_stats_device_index_bounds():
    """sm_arena_stats / sm_arena_reset_peak ignore out-of-range device slots."""
    lib = arena.library()
    out = (ctypes.c_uint64 * 8)(*([7] * 8))
    lib.sm_arena_stats(99, out)
    assert list(out) == [0] * 8
    lib.sm_arena_reset_peak(-1)
