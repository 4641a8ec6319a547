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


def test_torch_library_registration():
    """Every compute entry point of the C ABI is a torch.ops.ssl_mae operator with a
    schema (SURVEY.md §8(b) Registration); workspace / partial-size queries stay
    host-side.  Fake (meta) implementations propagate shapes without a GPU."""
    import torch
    from torch._subclasses.fake_tensor import FakeTensorMode
    from ssl_mae_amd import _lib, ops
    registered = set(ops.registered_ops())
    alias = {"layernorm_fwd": "layernorm", "dwconv_fwd": "dwconv", "gelu_fwd": "gelu", "fill": "fill_",
             "scale": "scale_", "dwconv_fused_fwd": "dwconv_fused", "pos_blend_fwd": "pos_blend",
             "dwconv_s2_bn_bwd": "dwconv_bn_bwd"}   # ssl_mae::dwconv_bn_bwd dispatches on stride
    internal = {"add",                       # not used by the step
                "bn_stats_from_partials",    # the statistics step inside ssl_mae::dwconv_fused
                "gemm_persistent",           # a host-side mode switch, no compute
                "gemm_tuning",               # A/B knobs of the GEMM dispatch (scripts only), no compute
                "attn_tuning",               # A/B switch of the attention backward's MFMA shape, no compute
                "calibrate_mfma"}            # bench.py's box calibration loop, not a step op
    for sym in _lib.exported_symbols():
        base = sym[3:]
        if base.endswith(("_workspace_bytes", "_partial_rows")) or base in internal:
            continue                          # host-side sizing queries
        name = alias.get(base, base)
        assert name in registered, (sym, name)
        assert str(getattr(torch.ops.ssl_mae, name).default._schema).startswith("ssl_mae::" + name)
    with FakeTensorMode():
        qkv = torch.empty(2 * 784, 3 * 384, dtype=torch.bfloat16)
        o, lse = ops.attn_fwd(qkv, 2, 784, 12, 32, 0.1, 123)
        assert o.shape == (2 * 784, 384) and lse.shape == (2, 12, 784)
        y, pre = ops.linear(torch.empty(64, 384, dtype=torch.bfloat16), torch.empty(1536, 384, dtype=torch.bfloat16),
                            torch.empty(1536), gelu=True)
        assert y.shape == pre.shape == (64, 1536)
        clip = torch.empty(2, 3, 8, 224, 224)
        col, geom = ops.stem_im2col(clip, torch.bfloat16)
        assert col.shape == (2 * 8 * 112 * 112, 32) and geom == (16, 112, 112)
        assert ops.patchify(clip).shape == (2, 8 * 28 * 28, 192)


def test_binding_argument_counts_match_header():
    """Every ctypes signature in _lib._SIGS has as many arguments as the header declares
    (a pointer missing from a binding shifts every later argument)."""
    from ssl_mae_amd import _lib
    src = open(os.path.join(ROOT, "include", "sm_api.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    decls = {}
    for m in re.finditer(r"\b(sm_[a-z0-9_]+)\s*\(([^)]*)\)\s*;", src):
        params = m.group(2).strip()
        decls[m.group(1)] = 0 if params in ("", "void") else params.count(",") + 1
    for name, (_, argtypes) in _lib._SIGS.items():
        assert name in decls, name
        assert len(argtypes) == decls[name], (name, len(argtypes), decls[name])


def test_gemm_tuning_defaults_match_the_library():
    """sm_gemm_tuning is host-side (no launch): every key kernels.GEMM_TUNING_KEYS names exists
    in the library, reads back the default kernels.gemm_tuning_nondefault compares against,
    and a set / reset round trip restores it; an unknown key is refused (-2)."""
    from ssl_mae_amd import _lib, build, kernels
    build.build()
    lib = ctypes.CDLL(_lib.LIB_PATH)
    fn = lib.sm_gemm_tuning
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
    assert list(kernels._GEMM_TUNING_DEFAULTS) == list(kernels.GEMM_TUNING_KEYS)
    for key, name in enumerate(kernels.GEMM_TUNING_KEYS):
        prev = ctypes.c_int(-12345)
        assert fn(key, 0, 0, ctypes.byref(prev)) == 0
        assert prev.value == kernels._GEMM_TUNING_DEFAULTS[name], name
        assert fn(key, 1, 7, ctypes.byref(prev)) == 0
        assert fn(key, 0, 0, ctypes.byref(prev)) == 0 and prev.value == 7
        assert fn(key, -1, 0, ctypes.byref(prev)) == 0
        assert fn(key, 0, 0, ctypes.byref(prev)) == 0 and prev.value == kernels._GEMM_TUNING_DEFAULTS[name]
    assert fn(len(kernels.GEMM_TUNING_KEYS), 0, 0, ctypes.byref(ctypes.c_int())) == -2
