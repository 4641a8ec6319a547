"""ctypes binding of libsslmae.so (the C ABI declared in include/sm_api.h).

The product path has no fallback: if the library is missing or fails to load,
every op raises.  `require()` is called by every kernel wrapper.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# SM_LIB_PATH: another build of the same library (same-box A/B of two builds, scripts/ab_lib.sh)
LIB_PATH = os.environ.get("SM_LIB_PATH") or os.path.join(_HERE, "libsslmae.so")

F32, BF16 = 0, 1
_DT = {torch.float32: F32, torch.bfloat16: BF16}

_c_i32 = ctypes.c_int
_c_i64 = ctypes.c_int64
_c_f32 = ctypes.c_float
_c_u64 = ctypes.c_uint64
_c_p = ctypes.c_void_p

# name -> (restype, argtypes)
_SIGS = {
    "sm_gemm_workspace_bytes": (_c_i64, [_c_i32, _c_i32, _c_i32, _c_i32]),
    "sm_gemm_persistent": (_c_i32, [_c_i32]),
    "sm_gemm_tuning": (_c_i32, [_c_i32, _c_i32, _c_i32, _c_p]),
    "sm_attn_tuning": (_c_i32, [_c_i32, _c_i32, _c_i32, _c_p]),
    "sm_calibrate_mfma": (_c_i32, [_c_i32, _c_i32, _c_i32, _c_p, _c_p, _c_p]),
    "sm_gemm": (_c_i32, [_c_i32, _c_i32, _c_i32, _c_i32, _c_i32, _c_i32, _c_i32, _c_p, _c_i64, _c_p, _c_i64,
                         _c_p, _c_i64, _c_p, _c_f32, _c_f32, _c_i32, _c_p, _c_p, _c_f32, _c_u64, _c_p, _c_i64,
                         _c_p, _c_i64, _c_p]),
    "sm_attn_fwd": (_c_i32, [_c_i32, _c_i32, _c_i32, _c_i32, _c_i32, _c_p, _c_p, _c_p, _c_f32, _c_f32, _c_u64,
                             _c_p]),
    "sm_attn_bwd_workspace_bytes": (_c_i64, [_c_i32] * 5),
    "sm_attn_bwd": (_c_i32, [_c_i32, _c_i32, _c_i32, _c_i32, _c_i32, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_f32,
                             _c_f32, _c_u64, _c_p]),
    "sm_layernorm_fwd": (_c_i32, [_c_i32, _c_i32, _c_i64, _c_i32, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_f32,
                                  _c_p]),
    "sm_layernorm_bwd_workspace_bytes": (_c_i64, [_c_i64, _c_i32]),
    "sm_layernorm_bwd": (_c_i32, [_c_i32, _c_i32, _c_i32, _c_i64, _c_i32, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p,
                                  _c_p, _c_p, _c_p, _c_p, _c_i64, _c_p]),
    "sm_layernorm_bwd_branch": (_c_i32, [_c_i32, _c_i32, _c_i32, _c_i64, _c_i32, _c_p, _c_p, _c_p, _c_p, _c_p,
                                         _c_p, _c_p, _c_p, _c_p, _c_p, _c_f32, _c_u64, _c_p, _c_i64, _c_p, _c_i64,
                                         _c_p]),
    "sm_bn_workspace_bytes": (_c_i64, [_c_i64, _c_i32]),
    "sm_bn_stats": (_c_i32, [_c_i32, _c_i64, _c_i32, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_f32, _c_f32, _c_i32,
                             _c_p, _c_i64, _c_p]),
    "sm_bn_apply": (_c_i32, [_c_i32, _c_i32, _c_i64, _c_i32, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_i32, _c_p,
                             _c_p, _c_i64, _c_p]),
    "sm_bn_bwd": (_c_i32, [_c_i32, _c_i32, _c_i64, _c_i32, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_i32, _c_p, _c_i64,
                           _c_p, _c_p, _c_p, _c_p, _c_i64, _c_p]),
    "sm_gelu_bwd": (_c_i32, [_c_i32, _c_i32, _c_i64, _c_i32, _c_p, _c_p, _c_p, _c_f32, _c_u64, _c_p]),
    "sm_dropout_bwd": (_c_i32, [_c_i32, _c_i64, _c_i32, _c_p, _c_p, _c_f32, _c_u64, _c_p, _c_i64, _c_p]),
    "sm_cast_dropout_bwd": (_c_i32, [_c_i64, _c_i32, _c_p, _c_p, _c_f32, _c_u64, _c_p, _c_i64, _c_p]),
    "sm_droppath_scale": (_c_i32, [_c_i32, _c_f32, _c_u64, _c_p, _c_p]),
    "sm_add": (_c_i32, [_c_i32, _c_i32, _c_i64, _c_p, _c_p, _c_p, _c_p]),
    "sm_cast": (_c_i32, [_c_i32, _c_i32, _c_i64, _c_p, _c_p, _c_p]),
    "sm_fill": (_c_i32, [_c_p, _c_i64, _c_f32, _c_p]),
    "sm_linear_dx_gelu": (_c_i32, [_c_i32] * 3 + [_c_p] * 5 + [_c_f32, _c_u64, _c_p]),
    "sm_gelu_fwd": (_c_i32, [_c_i32, _c_i64, _c_i32, _c_p, _c_p, _c_f32, _c_u64, _c_p]),
    "sm_linear_dw_bias_workspace_bytes": (_c_i64, [_c_i32, _c_i32, _c_i32]),
    "sm_linear_dw_bias": (_c_i32, [_c_i32, _c_i32, _c_i32, _c_p, _c_p, _c_p, _c_p, _c_i32, _c_p, _c_i64, _c_p]),
    "sm_linear_dw_bias_gelu": (_c_i32, [_c_i32, _c_i32, _c_i32, _c_p, _c_p, _c_f32, _c_u64, _c_p, _c_p, _c_i32, _c_p,
                                        _c_i64, _c_p]),
    "sm_linear_bn_stats_workspace_bytes": (_c_i64, [_c_i32, _c_i32]),
    "sm_linear_bn_stats": (_c_i32, [_c_i32, _c_i32, _c_i32, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_f32,
                                    _c_f32, _c_i32, _c_p, _c_i64, _c_p]),
    "sm_linear_bnin": (_c_i32, [_c_i32, _c_i32, _c_i32] + [_c_p] * 7 + [_c_p]),
    "sm_linear_bnin_bn_stats": (_c_i32, [_c_i32, _c_i32, _c_i32] + [_c_p] * 12 + [_c_f32, _c_f32, _c_i32, _c_p, _c_i64,
                                                                                  _c_p]),
    "sm_bn_apply_res_bn": (_c_i32, [_c_i32, _c_i32, _c_i64, _c_i32, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_i32, _c_p,
                                    _c_p, _c_p, _c_p, _c_p, _c_p, _c_i64, _c_p]),
    "sm_linear_se": (_c_i32, [_c_i32, _c_i32, _c_i32, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_i32, _c_p, _c_i32, _c_p,
                              _c_p]),
    "sm_linear_dw_se_workspace_bytes": (_c_i64, [_c_i32, _c_i32, _c_i32]),
    "sm_linear_dw_se": (_c_i32, [_c_i32, _c_i32, _c_i32, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_i32, _c_p, _c_i32,
                                 _c_p, _c_i32, _c_p, _c_i64, _c_p]),
    "sm_colsum_workspace_bytes": (_c_i64, [_c_i64, _c_i32]),
    "sm_colsum": (_c_i32, [_c_i32, _c_i64, _c_i32, _c_p, _c_p, _c_i32, _c_p, _c_i64, _c_p]),
    "sm_stem_im2col": (_c_i32, [_c_i32, _c_p, _c_i32, _c_i32, _c_i32, _c_i32, _c_i64, _c_i64, _c_i64, _c_i64,
                                _c_i64, _c_i32, _c_p, _c_p]),
    "sm_im2col3": (_c_i32, [_c_i32, _c_p, _c_i32, _c_i32, _c_i32, _c_i32, _c_i32, _c_p, _c_p]),
    "sm_col2im3": (_c_i32, [_c_i32, _c_p, _c_i32, _c_i32, _c_i32, _c_i32, _c_i32, _c_p, _c_p]),
    "sm_conv_wpack": (_c_i32, [_c_i32, _c_p, _c_p, _c_i32, _c_i32, _c_i32, _c_i32, _c_p]),
    "sm_stem_conv1_workspace_bytes": (_c_i64, []),
    "sm_stem_conv1_bn_stats": (_c_i32, [_c_p] + [_c_i32] * 4 + [_c_i64] * 5 + [_c_p] * 7
                               + [_c_f32, _c_f32, _c_i32, _c_p, _c_i64, _c_p]),
    "sm_stem_conv2_workspace_bytes": (_c_i64, [_c_i32]),
    "sm_stem_conv2_bn_stats": (_c_i32, [_c_p] + [_c_i32] * 3 + [_c_p] * 4 + [_c_i32] + [_c_p] * 7
                               + [_c_f32, _c_f32, _c_i32, _c_p, _c_i64, _c_p]),
    "sm_conv3x3_fwd": (_c_i32, [_c_p, _c_p, _c_p] + [_c_i32] * 5 + [_c_p]),
    "sm_conv3x3_fwd_bn_stats": (_c_i32, [_c_p, _c_p, _c_p] + [_c_i32] * 5 + [_c_p] * 5
                                + [_c_f32, _c_f32, _c_i32, _c_p, _c_i64, _c_p]),
    "sm_conv3x3_dgrad": (_c_i32, [_c_p, _c_p, _c_p] + [_c_i32] * 5 + [_c_p]),
    "sm_conv3x3_wgrad_workspace_bytes": (_c_i64, [_c_i32] * 5),
    "sm_conv3x3_wgrad": (_c_i32, [_c_p, _c_p, _c_p] + [_c_i32] * 6 + [_c_p, _c_i64, _c_p]),
    "sm_conv_wunpack_add": (_c_i32, [_c_p, _c_p, _c_i32, _c_i32, _c_i32, _c_i32, _c_p]),
    "sm_se_workspace_bytes": (_c_i64, [_c_i32, _c_i32, _c_i32]),
    "sm_se_fwd": (_c_i32, [_c_i32, _c_p] + [_c_p] * 4 + [_c_i32] * 5 + [_c_p] * 7 + [_c_i64, _c_p]),
    "sm_se_bwd": (_c_i32, [_c_i32, _c_p, _c_p] + [_c_p] * 4 + [_c_i32] * 5 + [_c_p] * 8 + [_c_i64, _c_p]),
    "sm_se_scale": (_c_i32, [_c_i32, _c_p] + [_c_p] * 4 + [_c_i32, _c_p, _c_p, _c_i32, _c_i32, _c_i32, _c_p]),
    "sm_se_bn_bwd_workspace_bytes": (_c_i64, [_c_i32, _c_i32, _c_i32]),
    "sm_se_bn_bwd": (_c_i32, [_c_i32, _c_p, _c_p] + [_c_p] * 4 + [_c_i32] * 5 + [_c_p] * 9 + [_c_p, _c_i64, _c_p]),
    "sm_dwconv_fused_partial_rows": (_c_i64, [_c_i32, _c_i32, _c_i32]),
    "sm_dwconv_fused_fwd": (_c_i32, [_c_i32] * 5 + [_c_p] * 5 + [_c_i32] + [_c_p] * 4),
    "sm_dwconv_fused_bwd_workspace_bytes": (_c_i64, [_c_i32] * 5),
    "sm_dwconv_fused_bwd": (_c_i32, [_c_i32] * 5 + [_c_p] * 6 + [_c_i32] + [_c_p] * 4 + [_c_i64, _c_p]),
    "sm_dwconv_bn_bwd_workspace_bytes": (_c_i64, [_c_i32] * 4),
    "sm_dwconv_bn_bwd": (_c_i32, [_c_i32] * 4 + [_c_p] * 6 + [_c_i32] + [_c_p] * 6 + [_c_i64, _c_p]),
    "sm_dwconv_s2_bn_bwd": (_c_i32, [_c_i32] * 4 + [_c_p] * 6 + [_c_i32] + [_c_p] * 6 + [_c_i64, _c_p]),
    "sm_bn_eval_params": (_c_i32, [_c_p, _c_p, _c_i32, _c_f32, _c_p, _c_p, _c_p]),
    "sm_segment_mean": (_c_i32, [_c_i32, _c_p, _c_i32, _c_i32, _c_i32, _c_p, _c_p]),
    "sm_segment_mean_bwd": (_c_i32, [_c_i32, _c_p, _c_i32, _c_i32, _c_i32, _c_p, _c_p]),
    "sm_bn_partials_workspace_bytes": (_c_i64, [_c_i32]),
    "sm_bn_stats_from_partials": (_c_i32, [_c_p, _c_i64, _c_i32, _c_i64] + [_c_p] * 5 + [_c_f32, _c_f32, _c_i32,
                                                                                       _c_p, _c_i64, _c_p]),
    "sm_dwconv_fwd": (_c_i32, [_c_i32, _c_p, _c_p, _c_p, _c_i32, _c_i32, _c_i32, _c_i32, _c_i32, _c_p]),
    "sm_dwconv_wgrad_workspace_bytes": (_c_i64, [_c_i32, _c_i32, _c_i32, _c_i32, _c_i32]),
    "sm_dwconv_bwd": (_c_i32, [_c_i32, _c_p, _c_p, _c_p, _c_p, _c_p, _c_i32, _c_i32, _c_i32, _c_i32, _c_i32, _c_p,
                               _c_i64, _c_p]),
    "sm_tube_mask": (_c_i32, [_c_p, _c_i32, _c_i32, _c_i32, _c_i32, _c_p, _c_p, _c_p]),
    "sm_pos_blend_fwd": (_c_i32, [_c_i32, _c_i32, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_i32, _c_i32, _c_i32,
                                  _c_i32, _c_p]),
    "sm_pos_blend_bwd": (_c_i32, [_c_i32, _c_i32, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_i32, _c_i32, _c_i32,
                                  _c_i32, _c_p]),
    "sm_loss_workspace_bytes": (_c_i64, [_c_i32, _c_i32, _c_i32]),
    "sm_mae_loss_fwd": (_c_i32, [_c_i32, _c_p, _c_p, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64, _c_p, _c_i32, _c_i32,
                                 _c_i32, _c_i32, _c_i32, _c_p, _c_p, _c_p, _c_i64, _c_p]),
    "sm_mae_loss_bwd": (_c_i32, [_c_i32, _c_p, _c_p, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64, _c_p, _c_i32, _c_i32,
                                 _c_i32, _c_i32, _c_i32, _c_p, _c_p, _c_p, _c_p]),
    "sm_patchify": (_c_i32, [_c_p, _c_i32, _c_i32, _c_i32, _c_i32, _c_i32, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64,
                             _c_i32, _c_p, _c_p]),
    "sm_unpatchify": (_c_i32, [_c_p, _c_i32, _c_i32, _c_i32, _c_i32, _c_i32, _c_i32, _c_p, _c_p]),
    "sm_scale": (_c_i32, [_c_p, _c_i64, _c_f32, _c_p]),
    "sm_gather_rows": (_c_i32, [_c_i32, _c_p, _c_p, _c_i64, _c_i32, _c_p, _c_p]),
    "sm_std_workspace_bytes": (_c_i64, []),
    "sm_std": (_c_i32, [_c_i32, _c_p, _c_i64, _c_p, _c_p, _c_i64, _c_p]),
    "sm_nonfinite": (_c_i32, [_c_p, _c_i64, _c_p, _c_p]),
    "sm_adamw": (_c_i32, [_c_p, _c_p, _c_p, _c_p, _c_p, _c_i64, _c_f32, _c_f32, _c_f32, _c_f32, _c_f32, _c_p, _c_p,
                          _c_i32, _c_p]),
    "sm_fedavg_weighted_sum": (_c_i32, [_c_i32, _c_p, _c_p, _c_i64, _c_p, _c_p]),
    "sm_fedavg_counters_max": (_c_i32, [_c_i32, _c_p, _c_i64, _c_p, _c_p]),
    "sm_frames_normalize": (_c_i32, [_c_p, _c_p, _c_i32, _c_i32, _c_i32, _c_i32, _c_p, _c_p, _c_i32, _c_p, _c_p]),
}

_lib = None


class KernelError(RuntimeError):
    pass


def load():
    """Load (not build) the shared library; raise if absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise KernelError(
            f"{LIB_PATH} is missing: the HIP kernels are not built (run __graft_entry__.build()). "
            "There is no CPU fallback on the product path.")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def exported_symbols():
    return list(_SIGS.keys())


def dt(t: torch.Tensor) -> int:
    try:
        return _DT[t.dtype]
    except KeyError:
        raise KernelError(f"unsupported dtype {t.dtype}") from None


def ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def call(name, *args):
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        raise KernelError(f"{name} failed with status {rc}")
    return rc


def query(name, *args):
    return getattr(load(), name)(*args)
