"""Device-memory arena for the training step (csrc/arena.cpp → libsmarena.so).

`install()` swaps PyTorch's caching allocator for the arena through the
pluggable-allocator hook; it has to run before the process's first CUDA
allocation (bench.py does it before torch.distributed / the model).  With the
arena in place the whole free HBM (minus `reserve_mib` for RCCL, code objects and
the runtime) is one best-fit, coalescing heap, which is what lets
`tiny_vit.auto_resident_stages` keep stage 0 resident at B = 256
(memory policy).  PyTorch's allocator statistics are not available
under a pluggable allocator: `stats()` / `max_memory_allocated()` read the
arena's own counters.
"""
import ctypes
import os

import torch

from .build import ARENA_LIB, build_arena

_state = {"lib": None}
_FIELDS = ("capacity", "in_use", "peak", "requests", "hipmalloc_requests", "free_blocks", "largest_free",
           "outside_bytes")


def _bind(path):
    lib = ctypes.CDLL(path)
    lib.sm_arena_stats.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_uint64)]
    lib.sm_arena_stats.restype = None
    lib.sm_arena_reset_peak.argtypes = [ctypes.c_int]
    lib.sm_arena_reset_peak.restype = None
    lib.sm_arena_attach.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64]
    lib.sm_arena_attach.restype = ctypes.c_int
    lib.sm_arena_alloc.argtypes = [ctypes.c_ssize_t, ctypes.c_int, ctypes.c_void_p]
    lib.sm_arena_alloc.restype = ctypes.c_void_p
    lib.sm_arena_free.argtypes = [ctypes.c_void_p, ctypes.c_ssize_t, ctypes.c_int, ctypes.c_void_p]
    lib.sm_arena_free.restype = None
    return lib


def library():
    """The arena library bound with ctypes (built in-tree if missing)."""
    if _state.get("raw") is None:
        _state["raw"] = _bind(build_arena())   # no-op when the library is newer than csrc/arena.cpp
    return _state["raw"]


def install(reserve_mib=None):
    """Make the arena PyTorch's CUDA allocator for this process.  Raises if a CUDA
    allocation already happened (the caching allocator cannot be swapped then)."""
    if _state["lib"] is not None:
        return
    if reserve_mib is not None:
        os.environ["SM_ARENA_RESERVE_MIB"] = str(int(reserve_mib))
    lib = library()
    alloc = torch.cuda.memory.CUDAPluggableAllocator(ARENA_LIB, "sm_arena_alloc", "sm_arena_free")
    torch.cuda.memory.change_current_allocator(alloc)
    _state["lib"] = lib
    _state["alloc"] = alloc


def active():
    return _state["lib"] is not None


def stats(device=None):
    """The arena's counters for `device` (bytes / counts, see csrc/arena.cpp)."""
    if device is None or (isinstance(device, torch.device) and device.index is None):
        dev = torch.cuda.current_device()
    else:
        dev = int(getattr(device, "index", device))
    out = (ctypes.c_uint64 * 8)()
    library().sm_arena_stats(dev, out)
    return dict(zip(_FIELDS, (int(v) for v in out)))


def capacity_gib(device=None):
    """Arena capacity in GiB (0 before its first allocation)."""
    return stats(device)["capacity"] / 2 ** 30


def max_memory_allocated(device=None):
    """torch.cuda.max_memory_allocated under the arena or the caching allocator."""
    if active():
        s = stats(device)
        return s["peak"] + s["outside_bytes"]
    return torch.cuda.max_memory_allocated(device)
