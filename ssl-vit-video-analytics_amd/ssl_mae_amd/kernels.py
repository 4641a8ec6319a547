"""Thin tensor-level wrappers over the C ABI (include/sm_api.h).

Each function allocates its outputs (torch caching allocator, current device),
launches on the current stream and returns tensors.  No CPU path exists: a
missing library or a non-CUDA tensor raises.
"""
import math

import torch

from . import _lib
from ._lib import call, dt, ptr, query, stream


def _chk(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise _lib.KernelError("ssl_mae_amd kernels need device tensors (no CPU fallback)")


def _ws(nbytes, device):
    return torch.empty(max(int(nbytes), 16), dtype=torch.uint8, device=device)


# ------------------------------------------------------------------ GEMM
def gemm(A, B, C, M, N, K, a_layout, b_layout, lda, ldb, ldc, bias=None, alpha=1.0, beta=0.0,
         gelu=False, aux=None, R=None, round_branch=False, drop_p=0.0, seed=0, row_scale=None, rows_per_group=1,
         gelu_bwd=False):
    _chk(A, B, C)
    ab = dt(A)
    if dt(B) != ab:
        raise _lib.KernelError("GEMM operands must share a dtype")
    nbytes = query("sm_gemm_workspace_bytes", ab, M, N, K)
    ws = _ws(nbytes, A.device) if nbytes else None
    epi = (1 if gelu else 0) | (2 if round_branch else 0) | (4 if gelu_bwd else 0)
    call("sm_gemm", ab, dt(C), a_layout, b_layout, M, N, K, ptr(A), lda, ptr(B), ldb, ptr(C), ldc, ptr(bias),
         float(alpha), float(beta), epi, ptr(aux), ptr(R), float(drop_p), int(seed) & ((1 << 64) - 1), ptr(row_scale),
         int(rows_per_group), ptr(ws), nbytes, stream())
    return C


def gemm_persistent(mode=-1):
    """Select the persistent (1) or one-tile-per-block (0) form of the plain bf16 forward /
    data-gradient GEMMs (bit-identical outputs); mode < 0 queries.  Returns the previous mode."""
    return int(query("sm_gemm_persistent", int(mode)))


GEMM_TUNING_KEYS = ("variant", "pp", "pp_min_n", "pp_max_k", "pp_rounds", "pp_rounds_small_k", "pp_rounds_mid_k",
                    "mf16_min_k", "dw384", "dw384_notr")


def gemm_tuning(key, value=None, reset=False):
    """A/B knob of the GEMM dispatch (sm_gemm_tuning; scripts/ only, the product path never
    sets one): returns the current value of `key` (GEMM_TUNING_KEYS), then stores `value`
    (or the default with reset=True)."""
    import ctypes
    k = GEMM_TUNING_KEYS.index(key)
    prev = ctypes.c_int(0)
    call("sm_gemm_tuning", k, -1 if reset else (1 if value is not None else 0), int(value or 0),
         ctypes.addressof(prev))
    return prev.value


_GEMM_TUNING_DEFAULTS = {"variant": 0, "pp": 1, "pp_min_n": 128, "pp_max_k": 384, "pp_rounds": -1,
                         "pp_rounds_small_k": 8, "pp_rounds_mid_k": 2, "mf16_min_k": 1 << 30,
                         "dw384": 1, "dw384_notr": 1}


def gemm_tuning_nondefault():
    """{key: value} of every GEMM knob not at its default (reported in bench.py's config)."""
    out = {}
    for k, d in _GEMM_TUNING_DEFAULTS.items():
        v = gemm_tuning(k)
        if v != d:
            out[k] = v
    return out


def calibrate_mfma(shape=32, iters=20000, blocks=None, device=None):
    """Bare bf16 MFMA loop on random register data (csrc/calib.hip), the box calibration of
    bench.py: shape 32 = v_mfma_f32_32x32x16_bf16, 16 = v_mfma_f32_16x16x32_bf16; `blocks`
    workgroups of 4 waves (default 2 per CU).  Returns (TFLOP/s, median in-kernel clock MHz,
    ms) over one timed launch after a warm-up launch."""
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    if blocks is None:
        blocks = 2 * torch.cuda.get_device_properties(dev).multi_processor_count
    stamps = torch.zeros(blocks, 2, dtype=torch.int64, device=dev)
    sink = torch.zeros(blocks * 256, dtype=torch.float32, device=dev)
    call("sm_calibrate_mfma", int(shape), max(1, int(iters) // 10), int(blocks), ptr(stamps), ptr(sink), stream())   # warm-up
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    call("sm_calibrate_mfma", int(shape), int(iters), int(blocks), ptr(stamps), ptr(sink), stream())
    e.record()
    e.synchronize()
    ms = s.elapsed_time(e)
    flop = 2.0 * 32 * 32 * 16 * 8 * iters * 4 * blocks    # 8 MFMAs (32x32x16 or 2x 16x16x32 pairs) per iter
    st = stamps.cpu()
    mem, real = st[:, 0].double(), st[:, 1].double()
    ok = real > 0
    mhz = float((mem[ok] / real[ok] * 100.0).median()) if ok.any() else None
    return flop / (ms * 1e-3) / 1e12, mhz, ms


def linear(x, w, bias=None, out_dtype=None, gelu=False, residual=None, round_branch=False, drop_p=0.0, seed=0,
           row_scale=None, rows_per_group=1):
    """y = residual + rs[row] * drop(act(x @ w^T + bias)); returns (y, pre-activation) with GELU."""
    M, K = x.shape
    N = w.shape[0]
    out = torch.empty((M, N), dtype=out_dtype or x.dtype, device=x.device)
    pre = torch.empty_like(out) if gelu else None
    gemm(x, w, out, M, N, K, 0, 0, K, K, N, bias=bias, gelu=gelu, aux=pre,
         beta=1.0 if residual is not None else 0.0, R=residual, round_branch=round_branch, drop_p=drop_p,
         seed=seed, row_scale=row_scale, rows_per_group=rows_per_group)
    return (out, pre) if gelu else out


def linear_dx(dy, w, out_dtype=None, residual=None, gelu_pre=None, drop_p=0.0, seed=0):
    """dx = dy @ w (+ residual);  dy [M,N], w [N,K].  gelu_pre: the input of a GELU (with
    dropout drop_p / seed on its output) that produced this Linear's input: returns the
    gradient w.r.t. that pre-activation, dx * keep/(1-p) * GELU'(gelu_pre), in the
    epilogue (no dh round trip, no separate gelu_bwd pass)."""
    M, N = dy.shape
    K = w.shape[1]
    out = torch.empty((M, K), dtype=out_dtype or dy.dtype, device=dy.device)
    if gelu_pre is not None:
        if gelu_pre.shape != out.shape or gelu_pre.dtype != out.dtype or residual is not None:
            raise _lib.KernelError("linear_dx: gelu_pre must match dx's shape/dtype (no residual)")
        gemm(dy, w, out, M, K, N, 0, 1, N, K, K, aux=gelu_pre.contiguous(), gelu_bwd=True, drop_p=drop_p, seed=seed)
        return out
    gemm(dy, w, out, M, K, N, 0, 1, N, K, K, beta=1.0 if residual is not None else 0.0, R=residual)
    return out


def linear_dx_gelu(dy, w, pre, drop_p=0.0, seed=0):
    """(dL/dpre, h) of y = dropout(GELU(pre)) @ w^T: dL/dpre = linear_dx(dy, w, gelu_pre=pre)
    and h = gelu(pre, drop_p, seed) (the fc2 weight gradient's operand) from one GEMM
    epilogue (sm_linear_dx_gelu): pre is read once, no recompute pass.  bf16 only."""
    _chk(dy, w, pre)
    M, N = dy.shape
    K = w.shape[1]
    if (dy.dtype != torch.bfloat16 or w.dtype != torch.bfloat16 or pre.dtype != torch.bfloat16
            or tuple(pre.shape) != (M, K) or w.shape[0] != N):
        raise _lib.KernelError("linear_dx_gelu: bf16 dy [M,N], w [N,K], pre [M,K]")
    dx = torch.empty((M, K), dtype=torch.bfloat16, device=dy.device)
    h = torch.empty_like(dx)
    call("sm_linear_dx_gelu", M, N, K, ptr(dy), ptr(w), ptr(pre), ptr(dx), ptr(h), float(drop_p), int(seed), stream())
    return dx, h


def linear_dw(dy, x, grad_sink, accumulate=True):
    """grad_sink[N,K] (+)= dy^T @ x   (fp32 sink; reduction over the M token rows)."""
    M, N = dy.shape
    K = x.shape[1]
    gemm(dy, x, grad_sink, N, K, M, 1, 1, N, K, K, beta=1.0 if accumulate else 0.0)
    return grad_sink


def linear_dw_bias(dy, x, grad_w, grad_b, gelu=None):
    """grad_w[N,K] += dy^T @ x' and grad_b[N] += sum over rows of dy.  bf16: one GEMM
    whose n0 == 0 blocks also sum dy (sm_linear_dw_bias); fp32 (parity): two ops.
    x' = x, or with gelu=(drop_p, seed) x' = dropout(GELU(x)) of the fc1 pre-activation
    x: formed in the GEMM's operand loads (sm_linear_dw_bias_gelu) when the weight
    gradient has one 256-row tile (N <= 256), else by the gelu kernel first (two
    m-tiles would activate every element twice; the recompute pass is cheaper)."""
    M, N = dy.shape
    K = x.shape[1]
    if gelu is not None:
        if (N <= 256 and dy.dtype == torch.bfloat16 and x.dtype == torch.bfloat16 and N % 8 == 0 and K % 8 == 0):
            _chk(dy, x, grad_w, grad_b)
            nbytes = query("sm_linear_dw_bias_workspace_bytes", M, N, K)
            ws = _ws(nbytes, dy.device)
            call("sm_linear_dw_bias_gelu", M, N, K, ptr(dy), ptr(x), float(gelu[0]), int(gelu[1]), ptr(grad_w),
                 ptr(grad_b), 1, ptr(ws), nbytes, stream())
            return grad_w
        return linear_dw_bias(dy, gelu_fwd(x, gelu[0], gelu[1]), grad_w, grad_b)
    if dy.dtype == torch.bfloat16 and x.dtype == torch.bfloat16 and N % 8 == 0 and K % 8 == 0:
        _chk(dy, x, grad_w, grad_b)
        nbytes = query("sm_linear_dw_bias_workspace_bytes", M, N, K)
        ws = _ws(nbytes, dy.device)
        call("sm_linear_dw_bias", M, N, K, ptr(dy), ptr(x), ptr(grad_w), ptr(grad_b), 1, ptr(ws), nbytes, stream())
        return grad_w
    linear_dw(dy, x, grad_w)
    colsum(dy, grad_b)
    return grad_w


def linear_bn_stats(x, w, running_mean=None, running_var=None, momentum=0.1, eps=1e-5, updates=1,
                    num_batches=None):
    """y = x @ w^T (bf16) and the train-mode BatchNorm statistics of y from the GEMM's
    epilogue (sm_linear_bn_stats; = linear + bn_stats without the read pass of y).
    Returns (y, mean, rstd)."""
    _chk(x, w)
    M, Kd = x.shape
    N = w.shape[0]
    if w.shape[1] != Kd or x.dtype != torch.bfloat16 or w.dtype != torch.bfloat16:
        raise _lib.KernelError("linear_bn_stats: bf16 x [M,K], w [N,K]")
    y = torch.empty((M, N), dtype=torch.bfloat16, device=x.device)
    mean = torch.empty(N, dtype=torch.float32, device=x.device)
    rstd = torch.empty(N, dtype=torch.float32, device=x.device)
    nbytes = query("sm_linear_bn_stats_workspace_bytes", M, N)
    ws = _ws(nbytes, x.device)
    call("sm_linear_bn_stats", M, N, Kd, ptr(x), ptr(w), ptr(y), ptr(mean), ptr(rstd), ptr(running_mean),
         ptr(running_var), ptr(num_batches), float(momentum), float(eps), int(updates), ptr(ws), nbytes, stream())
    return y, mean, rstd


def linear_bnin(a, act, w, bn=None, updates=1):
    """y [M,N] bf16 = x @ w^T with x = bf16(BN(a)) (act = (mean, rstd, weight, bias), no GELU)
    formed in the GEMM's A-operand loads (sm_linear_bnin; bit-identical to bn_apply +
    linear).  bn: also the train-mode BatchNorm statistics of y (sm_linear_bnin_bn_stats,
    = linear_bn_stats); returns y, or (y, mean, rstd) with bn."""
    _chk(a, w, *act[:4])
    M, Kd = a.shape
    N = w.shape[0]
    if w.shape[1] != Kd or a.dtype != torch.bfloat16 or w.dtype != torch.bfloat16 or act[4]:
        raise _lib.KernelError("linear_bnin: bf16 a [M,K], w [N,K], BatchNorm act without GELU")
    y = torch.empty((M, N), dtype=torch.bfloat16, device=a.device)
    if bn is None:
        call("sm_linear_bnin", M, N, Kd, ptr(a), *[ptr(t) for t in act[:4]], ptr(w), ptr(y), stream())
        return y
    running_mean, running_var, momentum, eps, num_batches = bn
    mean = torch.empty(N, dtype=torch.float32, device=a.device)
    rstd = torch.empty(N, dtype=torch.float32, device=a.device)
    nbytes = query("sm_linear_bn_stats_workspace_bytes", M, N)
    ws = _ws(nbytes, a.device)
    call("sm_linear_bnin_bn_stats", M, N, Kd, ptr(a), *[ptr(t) for t in act[:4]], ptr(w), ptr(y), ptr(mean),
         ptr(rstd), ptr(running_mean), ptr(running_var), ptr(num_batches), float(momentum), float(eps), int(updates),
         ptr(ws), nbytes, stream())
    return y, mean, rstd


def linear_se(a2, w, act, gate, hw):
    """y [M,N] bf16 = h3 @ w^T with h3 = se_scale(a2, gate, act) formed in the GEMM's
    A-operand loads (sm_linear_se; bit-identical to se_fwd's h3 + linear).  a2 [M,C] bf16,
    w [N,C] bf16, gate [M/hw, C] fp32, hw % 128 == 0, C % 64 == 0."""
    _chk(a2, w, gate)
    M, C = a2.shape
    N = w.shape[0]
    if w.shape[1] != C or gate.shape != (M // hw, C) or M % hw:
        raise _lib.KernelError("linear_se: shape mismatch")
    y = torch.empty((M, N), dtype=torch.bfloat16, device=a2.device)
    call("sm_linear_se", M, N, C, ptr(a2), ptr(w), *_act_args(act), ptr(gate.contiguous()), int(hw), ptr(y),
         stream())
    return y


def linear_dw_se(dy, a2, act, gate, hw, grad_sink, accumulate=True):
    """grad_sink[N,C] (+)= dy^T @ h3 with h3 = se_scale(a2, gate, act) formed in the GEMM's
    operand loads (sm_linear_dw_se; bit-identical to se_scale + linear_dw).  dy [M,N],
    a2 [M,C] bf16, gate [M/hw, C] fp32, hw % 64 == 0."""
    _chk(dy, a2, grad_sink)
    M, N = dy.shape
    C = a2.shape[1]
    if gate is None:          # B = the BatchNorm output act(a2) itself (the stem's BN2, no gate)
        hw = 1
    elif gate.shape != (M // hw, C) or M % hw:
        raise _lib.KernelError("linear_dw_se: gate shape mismatch")
    if a2.shape[0] != M or grad_sink.shape != (N, C):
        raise _lib.KernelError("linear_dw_se: shape mismatch")
    nbytes = query("sm_linear_dw_se_workspace_bytes", M, N, C)
    ws = _ws(nbytes, dy.device)
    call("sm_linear_dw_se", M, N, C, ptr(dy), ptr(a2), *_act_args(act),
         ptr(None if gate is None else gate.contiguous()), int(hw), ptr(grad_sink), 1 if accumulate else 0,
         ptr(ws), nbytes, stream())
    return grad_sink


def colsum(x, out, accumulate=True):
    M, C = x.shape
    nbytes = query("sm_colsum_workspace_bytes", M, C)
    ws = _ws(nbytes, x.device)
    call("sm_colsum", dt(x), M, C, ptr(x), ptr(out), 1 if accumulate else 0, ptr(ws), nbytes, stream())
    return out


# ------------------------------------------------------------------ attention
def attn_tuning(D, shape=None, reset=False):
    """MFMA shape of the bf16 attention backward for head dim D (sm_attn_tuning): 32 =
    v_mfma_f32_32x32x16_bf16, 16 = v_mfma_f32_16x16x32_bf16.  Returns the current shape,
    then stores `shape` (or the default with reset=True).  Tests and A/B scripts only."""
    import ctypes
    prev = ctypes.c_int(0)
    call("sm_attn_tuning", 0 if D == 64 else 1, -1 if reset else (1 if shape is not None else 0), int(shape or 0),
         ctypes.addressof(prev))
    return prev.value


def attn_fwd(qkv, N, L, H, D, drop_p=0.0, seed=0):
    _chk(qkv)
    out = torch.empty((N * L, H * D), dtype=qkv.dtype, device=qkv.device)
    lse = torch.empty((N, H, L), dtype=torch.float32, device=qkv.device)
    call("sm_attn_fwd", dt(qkv), N, L, H, D, ptr(qkv), ptr(out), ptr(lse), 1.0 / math.sqrt(D), float(drop_p),
         int(seed), stream())
    return out, lse


def attn_bwd(qkv, o, do, lse, N, L, H, D, drop_p=0.0, seed=0):
    _chk(qkv, o, do, lse)
    dqkv = torch.empty_like(qkv)
    ws = _ws(query("sm_attn_bwd_workspace_bytes", dt(qkv), N, L, H, D), qkv.device)   # Delta (+ scaled Q)
    call("sm_attn_bwd", dt(qkv), N, L, H, D, ptr(qkv), ptr(o), ptr(do), ptr(lse), ptr(ws), ptr(dqkv),
         1.0 / math.sqrt(D), float(drop_p), int(seed), stream())
    return dqkv


# ------------------------------------------------------------------ LayerNorm
def layernorm(x, gamma, beta, out_dtype=None, eps=1e-5):
    _chk(x)
    M, C = x.shape
    y = torch.empty((M, C), dtype=out_dtype or x.dtype, device=x.device)
    mean = torch.empty(M, dtype=torch.float32, device=x.device)
    rstd = torch.empty(M, dtype=torch.float32, device=x.device)
    call("sm_layernorm_fwd", dt(x), dt(y), M, C, ptr(x), ptr(gamma), ptr(beta), ptr(y), ptr(mean), ptr(rstd),
         float(eps), stream())
    return y, mean, rstd


def layernorm_recompute(x, gamma, beta, out_dtype, eps=1e-5):
    return layernorm(x, gamma, beta, out_dtype, eps)[0]


def layernorm_bwd(dy, x, mean, rstd, gamma, dgamma, dbeta, dres=None):
    M, C = x.shape
    dx = torch.empty_like(x)
    nbytes = query("sm_layernorm_bwd_workspace_bytes", M, C)
    ws = _ws(nbytes, x.device)
    call("sm_layernorm_bwd", dt(x), dt(dy), dt(dx), M, C, ptr(dy), ptr(x), ptr(mean), ptr(rstd), ptr(gamma),
         ptr(dx), ptr(dres), ptr(dgamma), ptr(dbeta), ptr(ws), nbytes, stream())
    return dx


def layernorm_bwd_branch(dy, x, mean, rstd, gamma, dgamma, dbeta, dres=None, drop_p=0.0, seed=0, row_scale=None,
                         rows_per_group=1):
    """layernorm_bwd plus the branch copy dxb = bf16(bf16(dx) * row_scale * dropout keep)
    (sm_layernorm_bwd_branch; = cast + dropout_bwd of dx).  Returns (dx, dxb)."""
    M, C = x.shape
    dx = torch.empty_like(x)
    dxb = torch.empty((M, C), dtype=torch.bfloat16, device=x.device)
    nbytes = query("sm_layernorm_bwd_workspace_bytes", M, C)
    ws = _ws(nbytes, x.device)
    call("sm_layernorm_bwd_branch", dt(x), dt(dy), dt(dx), M, C, ptr(dy), ptr(x), ptr(mean), ptr(rstd), ptr(gamma),
         ptr(dx), ptr(dres), ptr(dgamma), ptr(dbeta), ptr(dxb), float(drop_p), int(seed), ptr(row_scale),
         int(rows_per_group), ptr(ws), nbytes, stream())
    return dx, dxb


# ------------------------------------------------------------------ BatchNorm (train)
def bn_stats(x2d, running_mean=None, running_var=None, momentum=0.1, eps=1e-5, updates=1, num_batches=None):
    _chk(x2d)
    M, C = x2d.shape
    mean = torch.empty(C, dtype=torch.float32, device=x2d.device)
    rstd = torch.empty(C, dtype=torch.float32, device=x2d.device)
    nbytes = query("sm_bn_workspace_bytes", M, C)
    ws = _ws(nbytes, x2d.device)
    call("sm_bn_stats", dt(x2d), M, C, ptr(x2d), ptr(mean), ptr(rstd), ptr(running_mean), ptr(running_var),
         ptr(num_batches), float(momentum), float(eps), int(updates), ptr(ws), nbytes, stream())
    return mean, rstd


def bn_eval_params(bn):
    """(mean, rstd) of an eval-mode BatchNorm module from its running statistics."""
    C = bn.running_mean.numel()
    dev = bn.running_mean.device
    _chk(bn.running_mean)
    mean = torch.empty(C, dtype=torch.float32, device=dev)
    rstd = torch.empty(C, dtype=torch.float32, device=dev)
    call("sm_bn_eval_params", ptr(bn.running_mean), ptr(bn.running_var), C, float(bn.eps), ptr(mean), ptr(rstd),
         stream())
    return mean, rstd


def bn_apply(x2d, mean, rstd, w, b, gelu=False, out_dtype=None, residual=None, row_scale=None, rows_per_group=1,
             residual_bn=None):
    """residual_bn = (mean, rstd, weight, bias): the residual is stored before its own
    BatchNorm and enters as bf16(BN(residual)) (sm_bn_apply_res_bn)."""
    M, C = x2d.shape
    y = torch.empty((M, C), dtype=out_dtype or x2d.dtype, device=x2d.device)
    if residual_bn is not None:
        if residual is None:
            raise _lib.KernelError("bn_apply: residual_bn without a residual")
        call("sm_bn_apply_res_bn", dt(x2d), dt(y), M, C, ptr(x2d), ptr(mean), ptr(rstd), ptr(w), ptr(b), ptr(y),
             1 if gelu else 0, ptr(residual), *[ptr(t) for t in residual_bn[:4]], ptr(row_scale), int(rows_per_group),
             stream())
        return y
    call("sm_bn_apply", dt(x2d), dt(y), M, C, ptr(x2d), ptr(mean), ptr(rstd), ptr(w), ptr(b), ptr(y),
         1 if gelu else 0, ptr(residual), ptr(row_scale), int(rows_per_group), stream())
    return y


def bn_bwd(dy, x2d, mean, rstd, w, b, gelu, dw_sink, db_sink, row_scale=None, rows_per_group=1):
    M, C = x2d.shape
    dx = torch.empty_like(dy)
    nbytes = query("sm_bn_workspace_bytes", M, C)
    ws = _ws(nbytes, x2d.device)
    call("sm_bn_bwd", dt(x2d), dt(dy), M, C, ptr(dy), ptr(x2d), ptr(mean), ptr(rstd), ptr(w), ptr(b),
         1 if gelu else 0, ptr(row_scale), int(rows_per_group), ptr(dx), ptr(dw_sink), ptr(db_sink), ptr(ws),
         nbytes, stream())
    return dx


# ------------------------------------------------------------------ elementwise
def gelu(x, drop_p=0.0, seed=0):
    return gelu_fwd(x, drop_p, seed)


def gelu_fwd(x, drop_p=0.0, seed=0):
    y = torch.empty_like(x)
    call("sm_gelu_fwd", dt(x), x.numel(), x.shape[-1], ptr(x), ptr(y), float(drop_p), int(seed), stream())
    return y


def gelu_bwd(pre, dy, drop_p=0.0, seed=0):
    dx = torch.empty_like(dy)
    call("sm_gelu_bwd", dt(pre), dt(dy), dy.numel(), dy.shape[-1], ptr(pre), ptr(dy), ptr(dx), float(drop_p),
         int(seed), stream())
    return dx


def dropout_bwd(dy, drop_p=0.0, seed=0, row_scale=None, rows_per_group=1):
    dx = torch.empty_like(dy)
    call("sm_dropout_bwd", dt(dy), dy.numel(), dy.shape[-1], ptr(dy), ptr(dx), float(drop_p), int(seed),
         ptr(row_scale), int(rows_per_group), stream())
    return dx


def cast_dropout_bwd(dy, drop_p=0.0, seed=0, row_scale=None, rows_per_group=1):
    """bf16(bf16(dy) * row_scale * dropout keep) of an fp32 dy in one pass (= cast + dropout_bwd)."""
    _chk(dy)
    if dy.dtype != torch.float32:
        raise _lib.KernelError("cast_dropout_bwd takes an fp32 gradient")
    dx = torch.empty(dy.shape, dtype=torch.bfloat16, device=dy.device)
    call("sm_cast_dropout_bwd", dy.numel(), dy.shape[-1], ptr(dy), ptr(dx), float(drop_p), int(seed), ptr(row_scale),
         int(rows_per_group), stream())
    return dx


def droppath_scale(n, p, seed, device):
    out = torch.empty(n, dtype=torch.float32, device=device)
    call("sm_droppath_scale", int(n), float(p), int(seed), ptr(out), stream())
    return out


def add(a, b, out_dtype=None):
    o = torch.empty(b.shape, dtype=out_dtype or b.dtype, device=b.device)
    if dt(b) != dt(o):
        raise _lib.KernelError("add: b and out must share dtype")
    call("sm_add", dt(a), dt(o), o.numel(), ptr(a), ptr(b), ptr(o), stream())
    return o


def cast(a, dtype, out=None):
    o = out if out is not None else torch.empty(a.shape, dtype=dtype, device=a.device)
    call("sm_cast", dt(a), dt(o), a.numel(), ptr(a), ptr(o), stream())
    return o


def fill_(t, v):
    call("sm_fill", ptr(t), t.numel(), float(v), stream())
    return t


# ------------------------------------------------------------------ convolutions
def stem_im2col(clip, out_dtype, frames_view=None):
    """clip [B,3,T,H,W] (fp32, any strides) -> col [B*T*Ho*Wo, 32] (stride 2, pad 1)."""
    _chk(clip)
    if clip.dtype != torch.float32:
        clip = clip.float()
    if clip.dim() == 5:
        B, C, T, H, W = clip.shape
        sB, sC, sT, sH, sW = clip.stride()
    else:  # frames [N,3,H,W]
        B, C, H, W = clip.shape
        T = 1
        sB, sC, sH, sW = clip.stride()
        sT = 0
    Ho, Wo = (H + 1) // 2, (W + 1) // 2
    col = torch.empty((B * T * Ho * Wo, 32), dtype=out_dtype, device=clip.device)
    call("sm_stem_im2col", dt(col), ptr(clip), B, T, H, W, sB, sC, sT, sH, sW, 2, ptr(col), stream())
    return col, (B * T, Ho, Wo)


def stem_conv1_bn_stats(clip, wpack, running_mean=None, running_var=None, momentum=0.1, eps=1e-5, updates=1,
                        num_batches=None):
    """PatchEmbed conv1 (3->48, 3x3, stride 2, pad 1) straight from the fp32 clip [B,3,T,H,W]
    (or frames [N,3,H,W]; any strides) with bf16 order-0 packed weights [48][32], plus the
    train-mode BatchNorm statistics of its bf16 output (sm_stem_conv1_bn_stats;
    = stem_im2col + linear_bn_stats with no im2col buffer).  Returns (y, mean, rstd, (F, Ho, Wo))."""
    _chk(clip, wpack)
    if clip.dtype != torch.float32:
        clip = clip.float()
    if wpack.dtype != torch.bfloat16 or tuple(wpack.shape) != (48, 32) or not wpack.is_contiguous():
        raise _lib.KernelError("stem_conv1_bn_stats: wpack is contiguous bf16 [48][32]")
    if clip.dim() == 5:
        B, C, T, H, W = clip.shape
        sB, sC, sT, sH, sW = clip.stride()
    else:  # frames [N,3,H,W]
        B, C, H, W = clip.shape
        T = 1
        sB, sC, sH, sW = clip.stride()
        sT = 0
    Ho, Wo = (H + 1) // 2, (W + 1) // 2
    y = torch.empty((B * T * Ho * Wo, 48), dtype=torch.bfloat16, device=clip.device)
    mean = torch.empty(48, dtype=torch.float32, device=clip.device)
    rstd = torch.empty(48, dtype=torch.float32, device=clip.device)
    nbytes = query("sm_stem_conv1_workspace_bytes")
    ws = _ws(nbytes, clip.device)
    call("sm_stem_conv1_bn_stats", ptr(clip), B, T, H, W, sB, sC, sT, sH, sW, ptr(wpack), ptr(y), ptr(mean),
         ptr(rstd), ptr(running_mean), ptr(running_var), ptr(num_batches), float(momentum), float(eps), int(updates),
         ptr(ws), nbytes, stream())
    return y, mean, rstd, (B * T, Ho, Wo)


def stem_conv2_bn_stats(a1, act, wpack, F, H, W, running_mean=None, running_var=None, momentum=0.1, eps=1e-5,
                        updates=1, num_batches=None):
    """PatchEmbed conv2 over h1 = act(a1) (act = (mean, rstd, weight, bias, gelu) of BN1)
    plus the train-mode BatchNorm statistics of its bf16 output (sm_stem_conv2_bn_stats;
    = bn_apply + conv3x3_fwd_bn_stats with h1 never written).  a1 [F*H*W, 48] bf16, wpack
    order-1 [96, 432] bf16.  Returns (y [F*H*W, 96], mean, rstd)."""
    _chk(a1, wpack)
    _conv_chk(a1, 48)
    _conv_chk(wpack, 432)
    m, r, g, b, gelu = act
    y = torch.empty((F * H * W, 96), dtype=torch.bfloat16, device=a1.device)
    mean = torch.empty(96, dtype=torch.float32, device=a1.device)
    rstd = torch.empty(96, dtype=torch.float32, device=a1.device)
    nbytes = query("sm_stem_conv2_workspace_bytes", F)
    ws = _ws(nbytes, a1.device)
    call("sm_stem_conv2_bn_stats", ptr(a1), F, H, W, ptr(m), ptr(r), ptr(g), ptr(b), int(bool(gelu)), ptr(wpack),
         ptr(y), ptr(mean), ptr(rstd), ptr(running_mean), ptr(running_var), ptr(num_batches), float(momentum),
         float(eps), int(updates), ptr(ws), nbytes, stream())
    return y, mean, rstd


def im2col3(x, F, H, W, C, stride):
    Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
    col = torch.empty((F * Ho * Wo, 9 * C), dtype=x.dtype, device=x.device)
    call("sm_im2col3", dt(x), ptr(x), F, H, W, C, stride, ptr(col), stream())
    return col


def col2im3(dcol, F, H, W, C, stride):
    dx = torch.empty((F * H * W, C), dtype=dcol.dtype, device=dcol.device)
    call("sm_col2im3", dt(dcol), ptr(dcol), F, H, W, C, stride, ptr(dx), stream())
    return dx


def conv_wpack(w, Kpad, order, dtype):
    """w [Cout][Cin][3][3] fp32 -> packed [Cout][Kpad] (order 0 / 1) or [Cin][Kpad] (order 2)."""
    Cout, Cin = w.shape[0], w.shape[1]
    out = torch.empty((Cin if order == 2 else Cout, Kpad), dtype=dtype, device=w.device)
    call("sm_conv_wpack", dt(out), ptr(w), ptr(out), Cout, Cin, Kpad, order, stream())
    return out


def _conv_chk(t, C):
    if t.dtype != torch.bfloat16 or not t.is_contiguous() or t.shape[-1] != C:
        raise _lib.KernelError(f"conv3x3 operands are contiguous bf16 channels-last [pixels][{C}]")


def conv3x3_fwd(x, wpack, F, H, W, Cin, Cout):
    """Stem conv2 (3x3, stride 1, pad 1) over channels-last bf16 x [F*H*W, Cin] with
    order-1 packed weights [Cout][9*Cin]: implicit-im2col GEMM -> y [F*H*W, Cout] bf16."""
    _chk(x, wpack)
    _conv_chk(x, Cin)
    _conv_chk(wpack, 9 * Cin)
    y = torch.empty((F * H * W, Cout), dtype=torch.bfloat16, device=x.device)
    call("sm_conv3x3_fwd", ptr(x), ptr(wpack), ptr(y), F, H, W, Cin, Cout, stream())
    return y


def conv3x3_fwd_bn_stats(x, wpack, F, H, W, Cin, Cout, running_mean=None, running_var=None, momentum=0.1,
                         eps=1e-5, updates=1, num_batches=None):
    """conv3x3_fwd plus the train-mode BatchNorm statistics of y from the GEMM epilogue
    (sm_conv3x3_fwd_bn_stats; = conv3x3_fwd + bn_stats without the read pass of y).
    Returns (y, mean, rstd)."""
    _chk(x, wpack)
    _conv_chk(x, Cin)
    _conv_chk(wpack, 9 * Cin)
    P = F * H * W
    y = torch.empty((P, Cout), dtype=torch.bfloat16, device=x.device)
    mean = torch.empty(Cout, dtype=torch.float32, device=x.device)
    rstd = torch.empty(Cout, dtype=torch.float32, device=x.device)
    nbytes = query("sm_linear_bn_stats_workspace_bytes", P, Cout)
    ws = _ws(nbytes, x.device)
    call("sm_conv3x3_fwd_bn_stats", ptr(x), ptr(wpack), ptr(y), F, H, W, Cin, Cout, ptr(mean), ptr(rstd),
         ptr(running_mean), ptr(running_var), ptr(num_batches), float(momentum), float(eps), int(updates), ptr(ws),
         nbytes, stream())
    return y, mean, rstd


def conv3x3_dgrad(dy, wpack_t, F, H, W, Cin, Cout):
    """dL/dx of conv3x3_fwd from dy [F*H*W, Cout] and order-2 packed weights [Cin][9*Cout]."""
    _chk(dy, wpack_t)
    _conv_chk(dy, Cout)
    _conv_chk(wpack_t, 9 * Cout)
    dx = torch.empty((F * H * W, Cin), dtype=torch.bfloat16, device=dy.device)
    call("sm_conv3x3_dgrad", ptr(dy), ptr(wpack_t), ptr(dx), F, H, W, Cin, Cout, stream())
    return dx


def conv3x3_wgrad(dy, x, dw_sink, F, H, W, Cin, Cout, accumulate=True):
    """dw_sink [Cout][9*Cin] fp32 (+)= weight gradient of conv3x3_fwd (order-1 layout)."""
    _chk(dy, x, dw_sink)
    _conv_chk(dy, Cout)
    _conv_chk(x, Cin)
    if dw_sink.dtype != torch.float32 or dw_sink.shape != (Cout, 9 * Cin) or not dw_sink.is_contiguous():
        raise _lib.KernelError("conv3x3_wgrad sink is contiguous fp32 [Cout][9*Cin]")
    nbytes = query("sm_conv3x3_wgrad_workspace_bytes", F, H, W, Cin, Cout)
    ws = _ws(nbytes, dy.device)
    call("sm_conv3x3_wgrad", ptr(dy), ptr(x), ptr(dw_sink), 1 if accumulate else 0, F, H, W, Cin, Cout, ptr(ws),
         nbytes, stream())
    return dw_sink


def conv_wunpack_add(packed, grad, order):
    Cout, Cin = grad.shape[0], grad.shape[1]
    call("sm_conv_wunpack_add", ptr(packed), ptr(grad), Cout, Cin, packed.shape[1], order, stream())


def dwconv(x, w, F, H, W, C, stride):
    Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
    y = torch.empty((F * Ho * Wo, C), dtype=x.dtype, device=x.device)
    call("sm_dwconv_fwd", dt(x), ptr(x), ptr(w), ptr(y), F, H, W, C, stride, stream())
    return y


def dwconv_bwd(dy, x, w, dw_sink, F, H, W, C, stride, need_dx=True):
    dx = torch.empty_like(x) if need_dx else None
    nbytes = query("sm_dwconv_wgrad_workspace_bytes", F, H, W, C, stride)
    ws = _ws(nbytes, x.device)
    call("sm_dwconv_bwd", dt(x), ptr(dy), ptr(x), ptr(w), ptr(dx), ptr(dw_sink), F, H, W, C, stride, ptr(ws),
         nbytes, stream())
    return dx


def _act_args(act):
    """act = None or (mean, rstd, weight, bias, gelu): the BN(+GELU) folded into loads."""
    if act is None:
        return [None, None, None, None, 0]
    mean, rstd, w, b, gelu = act
    return [ptr(mean), ptr(rstd), ptr(w), ptr(b), 1 if gelu else 0]


def dwconv_fused(x, act, w, F, H, W, C, stride, bn_out=None, bn_updates=1):
    """y = dwconv3x3(act(x)) (bf16); with bn_out (a BatchNorm2d module) also its
    train-mode statistics of y (running stats updated bn_updates times): returns
    (y, mean, rstd) (or y)."""
    _chk(x)
    Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
    dev = x.device
    y = torch.empty((F * Ho * Wo, C), dtype=x.dtype, device=dev)
    part = None
    if bn_out is not None:
        rows = query("sm_dwconv_fused_partial_rows", F, H, stride)
        part = torch.empty((rows, 2, C), dtype=torch.float32, device=dev)
    a = _act_args(act)
    call("sm_dwconv_fused_fwd", F, H, W, C, stride, ptr(x), a[0], a[1], a[2], a[3], a[4], ptr(w), ptr(y), ptr(part),
         stream())
    if bn_out is None:
        return y
    mean = torch.empty(C, dtype=torch.float32, device=dev)
    rstd = torch.empty(C, dtype=torch.float32, device=dev)
    nbytes = query("sm_bn_partials_workspace_bytes", C)
    ws = _ws(nbytes, dev)
    call("sm_bn_stats_from_partials", ptr(part), part.shape[0], C, F * Ho * Wo, ptr(mean), ptr(rstd),
         ptr(bn_out.running_mean), ptr(bn_out.running_var), ptr(bn_out.num_batches_tracked),
         float(bn_out.momentum), float(bn_out.eps), int(bn_updates), ptr(ws), nbytes, stream())
    return y, mean, rstd


def dwconv_fused_bwd(dy, x, act, w, dw_sink, F, H, W, C, stride, need_dx=True):
    """dx = dL/d act(x), dw_sink += dL/dw for y = dwconv3x3(act(x)) (bf16)."""
    _chk(dy, x)
    dx = torch.empty_like(x) if need_dx else None
    nbytes = query("sm_dwconv_fused_bwd_workspace_bytes", F, H, W, C, stride)
    ws = _ws(nbytes, x.device)
    a = _act_args(act)
    call("sm_dwconv_fused_bwd", F, H, W, C, stride, ptr(dy), ptr(x), a[0], a[1], a[2], a[3], a[4], ptr(w), ptr(dx),
         ptr(dw_sink), ptr(ws), nbytes, stream())
    return dx


def dwconv_bn_bwd(dy, x, act, w, dw_sink, dg_sink, db_sink, F, H, W, C, stride=1):
    """y = dwconv3x3(act(x), stride 1 or 2), act = GELU(BN(x)) with batch statistics
    (act = (mean, rstd, gamma, beta, gelu)): returns dL/dx; dw_sink, dg_sink, db_sink
    += dL/dw, dL/dgamma, dL/dbeta (bf16).  F, H, W, C: the input's."""
    _chk(dy, x)
    dx = torch.empty_like(x)
    nbytes = query("sm_dwconv_bn_bwd_workspace_bytes", F, H, W, C)
    ws = _ws(nbytes, x.device)
    a = _act_args(act)
    call("sm_dwconv_s2_bn_bwd" if stride == 2 else "sm_dwconv_bn_bwd", F, H, W, C, ptr(dy), ptr(x), a[0], a[1], a[2], a[3], a[4], ptr(w), ptr(dx),
         ptr(dw_sink), ptr(dg_sink), ptr(db_sink), ptr(ws), nbytes, stream())
    return dx


def se_fwd(x, F, HW, C, w1, w2, act=None, want_y=True):
    """SELayer on h = act(x): returns (y = h * gate, pooled, relu(z1), gate)."""
    R = w1.shape[0]
    dev = x.device
    pooled = torch.empty((F, C), dtype=torch.float32, device=dev)
    h1 = torch.empty((F, R), dtype=torch.float32, device=dev)
    s = torch.empty((F, C), dtype=torch.float32, device=dev)
    y = torch.empty_like(x) if want_y else None
    nbytes = query("sm_se_workspace_bytes", F, HW, C)
    ws = _ws(nbytes, dev)
    call("sm_se_fwd", dt(x), ptr(x), *_act_args(act), F, HW, C, R, ptr(w1), ptr(w2), ptr(pooled), ptr(h1), ptr(s),
         ptr(y), ptr(ws), nbytes, stream())
    return y, pooled, h1, s


def se_scale(x, s, F, HW, C, act=None):
    y = torch.empty_like(x)
    call("sm_se_scale", dt(x), ptr(x), *_act_args(act), ptr(s), ptr(y), F, HW, C, stream())
    return y


def se_bwd(dy, x, F, HW, C, w1, w2, s, h1, act=None):
    R = w1.shape[0]
    dev = x.device
    dz2 = torch.empty((F, C), dtype=torch.float32, device=dev)
    dz1 = torch.empty((F, R), dtype=torch.float32, device=dev)
    dx = torch.empty_like(x)
    nbytes = query("sm_se_workspace_bytes", F, HW, C)
    ws = _ws(nbytes, dev)
    call("sm_se_bwd", dt(x), ptr(dy), ptr(x), *_act_args(act), F, HW, C, R, ptr(w1), ptr(w2), ptr(s), ptr(h1),
         ptr(dz2), ptr(dz1), ptr(dx), ptr(ws), nbytes, stream())
    return dx, dz2, dz1


def se_bn_bwd(dy, x, F, HW, C, w1, w2, s, h1, act, dw_sink, db_sink):
    """Fused backward of y = SE(GELU(BN(x))) with BN's batch statistics act = (mean,
    rstd, w, b, gelu): returns (dx, dz2, dz1) as se_bwd followed by bn_bwd on its dx;
    dw_sink / db_sink accumulate BN's weight / bias gradients."""
    _chk(dy, x)
    R = w1.shape[0]
    dev = x.device
    dz2 = torch.empty((F, C), dtype=torch.float32, device=dev)
    dz1 = torch.empty((F, R), dtype=torch.float32, device=dev)
    dx = torch.empty_like(x)
    nbytes = query("sm_se_bn_bwd_workspace_bytes", F, HW, C)
    ws = _ws(nbytes, dev)
    call("sm_se_bn_bwd", dt(x), ptr(dy), ptr(x), *_act_args(act), F, HW, C, R, ptr(w1), ptr(w2), ptr(s), ptr(h1),
         ptr(dz2), ptr(dz1), ptr(dx), ptr(dw_sink), ptr(db_sink), ptr(ws), nbytes, stream())
    return dx, dz2, dz1


# ------------------------------------------------------------------ MAE glue
def tube_mask(noise, T, n_mask, with_index=True):
    """noise [B,L] fp32 (device) -> mask uint8 [B,T,L], idx int32 [B*T*n_mask]."""
    _chk(noise)
    B, L = noise.shape
    mask = torch.empty((B, T, L), dtype=torch.uint8, device=noise.device)
    idx = torch.empty((B * T * n_mask,), dtype=torch.int32, device=noise.device) if with_index else None
    call("sm_tube_mask", ptr(noise), B, T, L, n_mask, ptr(mask), ptr(idx), stream())
    return mask, idx


def pos_blend(y, tpos, spos, tok, mask_u8, B, T, L, D, out_dtype):
    x = torch.empty((B * T * L, D), dtype=out_dtype, device=y.device)
    call("sm_pos_blend_fwd", dt(y), dt(x), ptr(y), ptr(tpos), ptr(spos), ptr(tok), ptr(mask_u8), ptr(x), B, T, L, D,
         stream())
    return x


def pos_blend_bwd(dx, mask_u8, y_dtype, dtpos, dspos, dtok, B, T, L, D):
    dy = torch.empty(dx.shape, dtype=y_dtype, device=dx.device)
    ws = torch.empty((2, B * T, D), dtype=torch.float32, device=dx.device)
    call("sm_pos_blend_bwd", dt(dx), dt(dy), ptr(dx), ptr(mask_u8), ptr(dy), ptr(dtpos), ptr(dspos), ptr(dtok),
         ptr(ws), B, T, L, D, stream())
    return dy


def _clip_args(clip):
    B, C, T, H, W = clip.shape
    return (B, T, H, W) + tuple(clip.stride())


def mae_loss_fwd(pred, clip, mask_u8, norm_pix=True):
    _chk(pred, clip, mask_u8)
    B, T, H, W, sB, sC, sT, sH, sW = _clip_args(clip)
    L = (H // 8) * (W // 8)
    loss = torch.empty((), dtype=torch.float32, device=pred.device)
    denom = torch.empty((1,), dtype=torch.float32, device=pred.device)
    nbytes = query("sm_loss_workspace_bytes", B, T, L)
    ws = _ws(nbytes, pred.device)
    call("sm_mae_loss_fwd", dt(pred), ptr(pred), ptr(clip), sB, sC, sT, sH, sW, ptr(mask_u8), B, T, H, W,
         1 if norm_pix else 0, ptr(loss), ptr(denom), ptr(ws), nbytes, stream())
    return loss, denom


def mae_loss_bwd(pred, clip, mask_u8, norm_pix, grad_out, denom):
    B, T, H, W, sB, sC, sT, sH, sW = _clip_args(clip)
    dpred = torch.empty_like(pred)
    g = grad_out.reshape(1).float().contiguous()
    call("sm_mae_loss_bwd", dt(pred), ptr(pred), ptr(clip), sB, sC, sT, sH, sW, ptr(mask_u8), B, T, H, W,
         1 if norm_pix else 0, ptr(g), ptr(denom), ptr(dpred), stream())
    return dpred


def patchify(imgs, p=8):
    _chk(imgs)
    x = imgs if imgs.dtype == torch.float32 else imgs.float()
    B, C, T, H, W = x.shape
    out = torch.empty((B, T * (H // p) * (W // p), p * p * C), dtype=torch.float32, device=x.device)
    call("sm_patchify", ptr(x), B, C, T, H, W, *x.stride(), p, ptr(out), stream())
    return out


def unpatchify(tokens, C, T, H, W, p=8):
    _chk(tokens)
    t = tokens.contiguous().float()
    B = t.shape[0]
    out = torch.empty((B, C, T, H, W), dtype=torch.float32, device=t.device)
    call("sm_unpatchify", ptr(t), B, C, T, H, W, p, ptr(out), stream())
    return out


def scale_(t, a):
    call("sm_scale", ptr(t), t.numel(), float(a), stream())
    return t


def gather_rows(src2d, idx):
    out = torch.empty((idx.numel(), src2d.shape[1]), dtype=src2d.dtype, device=src2d.device)
    call("sm_gather_rows", dt(src2d), ptr(src2d), ptr(idx), idx.numel(), src2d.shape[1], ptr(out), stream())
    return out


def std(x):
    out = torch.empty((), dtype=torch.float32, device=x.device)
    nbytes = query("sm_std_workspace_bytes")
    ws = _ws(nbytes, x.device)
    call("sm_std", dt(x), ptr(x), x.numel(), ptr(out), ptr(ws), nbytes, stream())
    return out


# ------------------------------------------------------------------ fine-tune head pooling
def segment_mean(x, G, R, C):
    """x [G*R, C] (or [G, R, C]) -> fp32 [G, C], mean over the R rows of each segment."""
    _chk(x)
    if not x.is_contiguous() or x.numel() != G * R * C:
        raise _lib.KernelError("segment_mean needs a contiguous [G][R][C] tensor")
    out = torch.empty((G, C), dtype=torch.float32, device=x.device)
    call("sm_segment_mean", dt(x), ptr(x), G, R, C, ptr(out), stream())
    return out


def segment_mean_bwd(dy, G, R, C, dtype):
    _chk(dy)
    if dy.dtype != torch.float32 or not dy.is_contiguous():
        raise _lib.KernelError("segment_mean_bwd takes the fp32 [G][C] gradient of segment_mean")
    dx = torch.empty((G * R, C), dtype=dtype, device=dy.device)
    call("sm_segment_mean_bwd", dt(dx), ptr(dy), G, R, C, ptr(dx), stream())
    return dx


# ------------------------------------------------------------------ optimizer
def nonfinite(g, flag):
    call("sm_nonfinite", ptr(g), g.numel(), ptr(flag), stream())


def adamw(p, g, m, v, lr, b1, b2, eps, wd, found_inf, step, shadow=None, advance_step=True):
    call("sm_adamw", ptr(p), ptr(g), ptr(m), ptr(v), ptr(shadow), p.numel(), float(lr), float(b1), float(b2),
         float(eps), float(wd), ptr(found_inf), ptr(step), 1 if advance_step else 0, stream())


# ------------------------------------------------------------------ federated averaging
def fedavg_weighted_sum(bufs, weights, out=None):
    """out = sum_j bufs[j] * weights[j] in client order (fed_loop.py:46-49), bit-exact.
    bufs: equal-length contiguous fp32 device tensors; weights: fp32-representable floats."""
    import ctypes
    if not bufs:
        raise _lib.KernelError("fedavg_weighted_sum needs at least one client buffer")
    _chk(*bufs)
    if len(weights) != len(bufs):
        raise _lib.KernelError(f"fedavg_weighted_sum: {len(bufs)} client buffers but {len(weights)} weights")
    n = bufs[0].numel()
    for b in bufs:
        if b.dtype != torch.float32 or b.numel() != n or not b.is_contiguous() or b.device != bufs[0].device:
            raise _lib.KernelError("fedavg client buffers must be contiguous fp32 of one length on one device")
    if out is None:
        out = torch.empty_like(bufs[0])
    k = len(bufs)
    ptrs = (ctypes.c_void_p * k)(*[b.data_ptr() for b in bufs])
    ws = (ctypes.c_float * k)(*[float(w) for w in weights])
    call("sm_fedavg_weighted_sum", k, ctypes.cast(ptrs, ctypes.c_void_p), ctypes.cast(ws, ctypes.c_void_p), n,
         ptr(out), stream())
    return out


def fedavg_counters_max(bufs, out=None):
    """out = elementwise max over clients of int64 counters (fed_loop.py:52-55)."""
    import ctypes
    if not bufs:
        raise _lib.KernelError("fedavg_counters_max needs at least one client buffer")
    _chk(*bufs)
    n = bufs[0].numel()
    for b in bufs:
        if b.dtype != torch.int64 or b.numel() != n or not b.is_contiguous() or b.device != bufs[0].device:
            raise _lib.KernelError("fedavg counters must be contiguous int64 of one length on one device")
    if out is None:
        out = torch.empty_like(bufs[0])
    k = len(bufs)
    ptrs = (ctypes.c_void_p * k)(*[b.data_ptr() for b in bufs])
    call("sm_fedavg_counters_max", k, ctypes.cast(ptrs, ctypes.c_void_p), n, ptr(out), stream())
    return out


# ------------------------------------------------------------------ clip input pipeline
def frames_normalize(frames, mean, std, bgr_swap=True, valid=None, out=None):
    """uint8 [B,T,H,W,3] decoded frames -> fp32 [B,3,T,H,W] normalised clip
    (train_ssl_mae.py:137-141 transform + mae_loader.py:70-77 BGR swap / permute)."""
    import ctypes
    _chk(frames, valid)
    if frames.dtype != torch.uint8 or frames.dim() != 5 or frames.shape[-1] != 3 or not frames.is_contiguous():
        raise _lib.KernelError("frames must be contiguous uint8 [B,T,H,W,3]")
    B, T, H, W, _ = frames.shape
    if valid is not None and (valid.dtype not in (torch.uint8, torch.bool) or valid.numel() != B):
        raise _lib.KernelError("valid must be uint8/bool [B]")
    if out is None:
        out = torch.empty((B, 3, T, H, W), dtype=torch.float32, device=frames.device)
    m = (ctypes.c_float * 3)(*[float(x) for x in mean])
    s = (ctypes.c_float * 3)(*[float(x) for x in std])
    call("sm_frames_normalize", ptr(frames), ptr(valid), B, T, H, W, ctypes.cast(m, ctypes.c_void_p),
         ctypes.cast(s, ctypes.c_void_p), 1 if bgr_swap else 0, ptr(out), stream())
    return out
