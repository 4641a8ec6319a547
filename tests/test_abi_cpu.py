"""CPU-side checks of the C ABI: the library builds/loads and exports every symbol
declared in include/sm_api.h (no compute calls without a GPU)."""
import ctypes
import os
import re

import pytest

from conftest import ROOT


def _declared():
    src = open(os.path.join(ROOT, "include", "sm_api.h")).read()
    return sorted(set(re.findall(r"\b(sm_[a-z0-9_]+)\s*\(", src)))


def test_header_and_binding_agree():
    from ssl_mae_amd import _lib
    assert sorted(_lib.exported_symbols()) == _declared()


def test_library_exports_every_declared_symbol():
    from ssl_mae_amd import _lib, build
    build.build()
    lib = ctypes.CDLL(_lib.LIB_PATH)
    for name in _declared():
        assert hasattr(lib, name), name
    _lib.load()


def test_no_cpu_fallback():
    import torch
    from ssl_mae_amd import kernels
    with pytest.raises(Exception):
        kernels.layernorm(torch.zeros(4, 8), torch.ones(8), torch.zeros(8))
