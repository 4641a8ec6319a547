"""PyTorch custom-op registration of the HIP kernels: namespace `ssl_mae`.

SURVEY.md §8(b) "Registration": every C-ABI entry point of libsslmae.so
(include/sm_api.h) is a `torch.ops.ssl_mae.*` operator with a schema (mutated
arguments annotated `Tensor(a!)`), a CUDA implementation that calls the C ABI on
the current stream (kernels.py), and a fake (meta) implementation for shape
propagation, so the ops are visible to the dispatcher, to `torch.compile` tracing
and to FakeTensor.  The differentiable primitives also carry
`register_autograd` formulas over the same kernels:

    attn_fwd     (tiny_vit.py:103 SDPA; decoder MHA core)  -> attn_bwd
    layernorm    (tiny_vit.py:112,115; decoder norms)      -> layernorm_bwd
    linear       (every nn.Linear / 1x1 conv, plain form)   -> linear_dx / linear_dw / GEMM bias sum
    gelu         (exact erf GELU)                           -> gelu_bwd
    mae_loss_fwd (train_ssl_mae.py:72-84)                   -> mae_loss_bwd
    patchify     (train_ssl_mae.py:26-31)                   -> unpatchify
    segment_mean (fine-tune pooling)                        -> segment_mean_bwd

The Python functions below keep kernels.py's signatures (composite arguments -- a
BatchNorm module, a folded (mean, rstd, w, b, gelu) activation -- are expanded
into tensors here), so the model code calls `ops.<name>` and every kernel launch
of the training step goes through the dispatcher.  The fused training-step
Functions (functions.py) stay torch.autograd.Function, which the survey's
registration row allows, because their backward writes weight gradients straight
into the flat fp32 gradient buffer (optim.FlatParams).
"""
import torch

from . import kernels as _K

_M64 = (1 << 64) - 1


def _s64(seed):
    """uint64 counter-RNG seed -> the schema's signed int."""
    u = int(seed) & _M64
    return u - (1 << 64) if u >= (1 << 63) else u


def _u64(s):
    return int(s) & _M64


def _op(name, schema, mutates=()):
    def deco(impl):
        return torch.library.custom_op(f"ssl_mae::{name}", impl, mutates_args=tuple(mutates), schema=schema)
    return deco


def _none(*a, **k):
    return None


def _e(like, dtype=None):
    return torch.empty(0, dtype=dtype or torch.float32, device=like.device)


# ============================================================================ GEMM
@_op("gemm", "(Tensor A, Tensor B, Tensor(a!) C, int M, int N, int K, int a_layout, int b_layout, int lda, "
             "int ldb, int ldc, Tensor? bias, float alpha, float beta, bool gelu, Tensor(b!)? aux, Tensor? R, "
             "bool round_branch, float drop_p, int seed, Tensor? row_scale, int rows_per_group) -> ()", ("C", "aux"))
def _gemm(A, B, C, M, N, K, a_layout, b_layout, lda, ldb, ldc, bias, alpha, beta, gelu, aux, R, round_branch, drop_p,
          seed, row_scale, rows_per_group):
    _K.gemm(A, B, C, M, N, K, a_layout, b_layout, lda, ldb, ldc, bias, alpha, beta, gelu, aux, R, round_branch,
            drop_p, _u64(seed), row_scale, rows_per_group)


_gemm.register_fake(_none)


def gemm(A, B, C, M, N, K, a_layout, b_layout, lda, ldb, ldc, bias=None, alpha=1.0, beta=0.0, gelu=False, aux=None,
         R=None, round_branch=False, drop_p=0.0, seed=0, row_scale=None, rows_per_group=1):
    torch.ops.ssl_mae.gemm(A, B, C, M, N, K, a_layout, b_layout, lda, ldb, ldc, bias, float(alpha), float(beta),
                           bool(gelu), aux, R, bool(round_branch), float(drop_p), _s64(seed), row_scale,
                           int(rows_per_group))
    return C


@_op("linear", "(Tensor x, Tensor w, Tensor? bias, ScalarType? out_dtype, bool gelu, Tensor? residual, "
               "bool round_branch, float drop_p, int seed, Tensor? row_scale, int rows_per_group) -> (Tensor, Tensor)")
def _linear(x, w, bias, out_dtype, gelu, residual, round_branch, drop_p, seed, row_scale, rows_per_group):
    r = _K.linear(x, w, bias, out_dtype, gelu, residual, round_branch, drop_p, _u64(seed), row_scale,
                  rows_per_group)
    return r if gelu else (r, _e(x))


@_linear.register_fake
def _(x, w, bias, out_dtype, gelu, residual, round_branch, drop_p, seed, row_scale, rows_per_group):
    y = x.new_empty((x.shape[0], w.shape[0]), dtype=out_dtype or x.dtype)
    return y, (torch.empty_like(y) if gelu else x.new_empty(0, dtype=torch.float32))


def _linear_ctx(ctx, inputs, output):
    x, w, bias, out_dtype, gelu, residual, round_branch, drop_p, seed, row_scale, rows_per_group = inputs
    ctx.plain = not gelu and residual is None and drop_p == 0.0 and row_scale is None
    ctx.has_bias = bias is not None
    ctx.save_for_backward(x, w)


def _linear_bwd(ctx, dy, dpre):
    if not ctx.plain:
        raise NotImplementedError("ssl_mae::linear autograd covers the plain form y = x w^T + b; "
                                  "epilogue variants are differentiated by the fused Functions")
    x, w = ctx.saved_tensors
    dy = dy.to(x.dtype).contiguous()
    dx = linear_dx(dy, w) if ctx.needs_input_grad[0] else None
    dw = linear_dw(dy, x, torch.zeros(w.shape, dtype=torch.float32, device=w.device)).to(w.dtype)
    db = None
    if ctx.has_bias:
        M, N = dy.shape
        ones = fill_(torch.empty(M, dtype=torch.float32, device=dy.device), 1.0)
        db = gemm(ones, dy.float(), torch.empty(N, dtype=torch.float32, device=dy.device), 1, N, M, 0, 1, M, N, N)
    return dx, dw, db, None, None, None, None, None, None, None, None


_linear.register_autograd(_linear_bwd, setup_context=_linear_ctx)


def linear(x, w, bias=None, out_dtype=None, gelu=False, residual=None, round_branch=False, drop_p=0.0, seed=0,
           row_scale=None, rows_per_group=1):
    y, pre = torch.ops.ssl_mae.linear(x, w, bias, out_dtype, bool(gelu), residual, bool(round_branch),
                                      float(drop_p), _s64(seed), row_scale, int(rows_per_group))
    return (y, pre) if gelu else y


@_op("linear_dx", "(Tensor dy, Tensor w, ScalarType? out_dtype, Tensor? residual, Tensor? gelu_pre, float drop_p, "
                  "int seed) -> Tensor")
def _linear_dx(dy, w, out_dtype, residual, gelu_pre, drop_p, seed):
    return _K.linear_dx(dy, w, out_dtype, residual, gelu_pre, drop_p, _u64(seed))


@_linear_dx.register_fake
def _(dy, w, out_dtype, residual, gelu_pre, drop_p, seed):
    return dy.new_empty((dy.shape[0], w.shape[1]), dtype=out_dtype or dy.dtype)


def linear_dx(dy, w, out_dtype=None, residual=None, gelu_pre=None, drop_p=0.0, seed=0):
    return torch.ops.ssl_mae.linear_dx(dy, w, out_dtype, residual, gelu_pre, float(drop_p), _s64(seed))


@_op("linear_dx_gelu", "(Tensor dy, Tensor w, Tensor pre, float drop_p, int seed) -> (Tensor, Tensor)")
def _linear_dx_gelu(dy, w, pre, drop_p, seed):
    return _K.linear_dx_gelu(dy, w, pre, drop_p, _u64(seed))


@_linear_dx_gelu.register_fake
def _(dy, w, pre, drop_p, seed):
    return pre.new_empty(pre.shape), pre.new_empty(pre.shape)


def linear_dx_gelu(dy, w, pre, drop_p=0.0, seed=0):
    """fc2 dX through dropout(GELU(pre)) + h = dropout(GELU(pre)) as a side output."""
    return torch.ops.ssl_mae.linear_dx_gelu(dy, w, pre, float(drop_p), _s64(seed))


@_op("linear_dw", "(Tensor dy, Tensor x, Tensor(a!) grad_sink, bool accumulate) -> ()", ("grad_sink",))
def _linear_dw(dy, x, grad_sink, accumulate):
    _K.linear_dw(dy, x, grad_sink, accumulate)


_linear_dw.register_fake(_none)


def linear_dw(dy, x, grad_sink, accumulate=True):
    torch.ops.ssl_mae.linear_dw(dy, x, grad_sink, bool(accumulate))
    return grad_sink


@_op("linear_dw_bias", "(Tensor dy, Tensor x, Tensor(a!) grad_w, Tensor(b!) grad_b) -> ()", ("grad_w", "grad_b"))
def _linear_dw_bias(dy, x, grad_w, grad_b):
    _K.linear_dw_bias(dy, x, grad_w, grad_b)


_linear_dw_bias.register_fake(_none)


def linear_dw_bias(dy, x, grad_w, grad_b, gelu=None):
    if gelu is not None:
        torch.ops.ssl_mae.linear_dw_bias_gelu(dy, x, grad_w, grad_b, float(gelu[0]), _s64(gelu[1]))
    else:
        torch.ops.ssl_mae.linear_dw_bias(dy, x, grad_w, grad_b)
    return grad_w


@_op("linear_dw_bias_gelu", "(Tensor dy, Tensor pre, Tensor(a!) grad_w, Tensor(b!) grad_b, float drop_p, "
                            "int seed) -> ()", ("grad_w", "grad_b"))
def _linear_dw_bias_gelu(dy, pre, grad_w, grad_b, drop_p, seed):
    _K.linear_dw_bias(dy, pre, grad_w, grad_b, gelu=(drop_p, _u64(seed)))


_linear_dw_bias_gelu.register_fake(_none)


@_op("colsum", "(Tensor x, Tensor(a!) out, bool accumulate) -> ()", ("out",))
def _colsum(x, out, accumulate):
    _K.colsum(x, out, accumulate)


_colsum.register_fake(_none)


def colsum(x, out, accumulate=True):
    torch.ops.ssl_mae.colsum(x, out, bool(accumulate))
    return out


# ============================================================================ attention
@_op("attn_fwd", "(Tensor qkv, int N, int L, int H, int D, float drop_p, int seed) -> (Tensor, Tensor)")
def _attn_fwd(qkv, N, L, H, D, drop_p, seed):
    return _K.attn_fwd(qkv, N, L, H, D, drop_p, _u64(seed))


@_attn_fwd.register_fake
def _(qkv, N, L, H, D, drop_p, seed):
    return qkv.new_empty((N * L, H * D)), qkv.new_empty((N, H, L), dtype=torch.float32)


def _attn_ctx(ctx, inputs, output):
    qkv, N, L, H, D, drop_p, seed = inputs
    ctx.args = (N, L, H, D, drop_p, seed)
    ctx.save_for_backward(qkv, output[0], output[1])


def _attn_bwd_formula(ctx, do, dlse):
    qkv, o, lse = ctx.saved_tensors
    N, L, H, D, drop_p, seed = ctx.args
    return attn_bwd(qkv, o, do.to(qkv.dtype).contiguous(), lse, N, L, H, D, drop_p, _u64(seed)), \
        None, None, None, None, None, None


_attn_fwd.register_autograd(_attn_bwd_formula, setup_context=_attn_ctx)


def attn_fwd(qkv, N, L, H, D, drop_p=0.0, seed=0):
    return torch.ops.ssl_mae.attn_fwd(qkv, N, L, H, D, float(drop_p), _s64(seed))


@_op("attn_bwd", "(Tensor qkv, Tensor o, Tensor do, Tensor lse, int N, int L, int H, int D, float drop_p, "
                 "int seed) -> Tensor")
def _attn_bwd(qkv, o, do, lse, N, L, H, D, drop_p, seed):
    return _K.attn_bwd(qkv, o, do, lse, N, L, H, D, drop_p, _u64(seed))


_attn_bwd.register_fake(lambda qkv, *a: torch.empty_like(qkv))


def attn_bwd(qkv, o, do, lse, N, L, H, D, drop_p=0.0, seed=0):
    return torch.ops.ssl_mae.attn_bwd(qkv, o, do, lse, N, L, H, D, float(drop_p), _s64(seed))


# ============================================================================ LayerNorm
@_op("layernorm", "(Tensor x, Tensor gamma, Tensor beta, ScalarType? out_dtype, float eps) -> (Tensor, Tensor, Tensor)")
def _layernorm(x, gamma, beta, out_dtype, eps):
    return _K.layernorm(x, gamma, beta, out_dtype, eps)


@_layernorm.register_fake
def _(x, gamma, beta, out_dtype, eps):
    M = x.shape[0]
    return (x.new_empty(x.shape, dtype=out_dtype or x.dtype), x.new_empty(M, dtype=torch.float32),
            x.new_empty(M, dtype=torch.float32))


def _ln_ctx(ctx, inputs, output):
    x, gamma, beta, out_dtype, eps = inputs
    ctx.save_for_backward(x, gamma, output[1], output[2])


def _ln_bwd(ctx, dy, dmean, drstd):
    x, gamma, mean, rstd = ctx.saved_tensors
    dg = torch.zeros(gamma.shape, dtype=torch.float32, device=x.device)
    db = torch.zeros(gamma.shape, dtype=torch.float32, device=x.device)
    dx = layernorm_bwd(dy.contiguous(), x, mean, rstd, gamma, dg, db)
    return dx, dg, db, None, None


_layernorm.register_autograd(_ln_bwd, setup_context=_ln_ctx)


def layernorm(x, gamma, beta, out_dtype=None, eps=1e-5):
    return torch.ops.ssl_mae.layernorm(x, gamma, beta, out_dtype, float(eps))


@_op("layernorm_bwd", "(Tensor dy, Tensor x, Tensor mean, Tensor rstd, Tensor gamma, Tensor(a!) dgamma, "
                      "Tensor(b!) dbeta, Tensor? dres) -> Tensor", ("dgamma", "dbeta"))
def _layernorm_bwd(dy, x, mean, rstd, gamma, dgamma, dbeta, dres):
    return _K.layernorm_bwd(dy, x, mean, rstd, gamma, dgamma, dbeta, dres)


_layernorm_bwd.register_fake(lambda dy, x, *a: torch.empty_like(x))


def layernorm_bwd(dy, x, mean, rstd, gamma, dgamma, dbeta, dres=None):
    return torch.ops.ssl_mae.layernorm_bwd(dy, x, mean, rstd, gamma, dgamma, dbeta, dres)


@_op("layernorm_bwd_branch", "(Tensor dy, Tensor x, Tensor mean, Tensor rstd, Tensor gamma, Tensor(a!) dgamma, "
                             "Tensor(b!) dbeta, Tensor? dres, float drop_p, int seed, Tensor? row_scale, "
                             "int rows_per_group) -> (Tensor, Tensor)", ("dgamma", "dbeta"))
def _layernorm_bwd_branch(dy, x, mean, rstd, gamma, dgamma, dbeta, dres, drop_p, seed, row_scale, rows_per_group):
    return _K.layernorm_bwd_branch(dy, x, mean, rstd, gamma, dgamma, dbeta, dres, drop_p, _u64(seed), row_scale,
                                   rows_per_group)


_layernorm_bwd_branch.register_fake(
    lambda dy, x, *a: (torch.empty_like(x), torch.empty(x.shape, dtype=torch.bfloat16, device=x.device)))


def layernorm_bwd_branch(dy, x, mean, rstd, gamma, dgamma, dbeta, dres=None, drop_p=0.0, seed=0, row_scale=None,
                         rows_per_group=1):
    """LayerNorm backward + the block branch's bf16 copy of dx with the branch's dropout /
    DropPath backward applied (one pass over dx instead of three)."""
    return torch.ops.ssl_mae.layernorm_bwd_branch(dy, x, mean, rstd, gamma, dgamma, dbeta, dres, float(drop_p),
                                                  _s64(seed), row_scale, int(rows_per_group))


# ============================================================================ BatchNorm
@_op("bn_stats", "(Tensor x, Tensor(a!)? running_mean, Tensor(b!)? running_var, float momentum, float eps, "
                 "int updates, Tensor(c!)? num_batches_tracked) -> (Tensor, Tensor)",
     ("running_mean", "running_var", "num_batches_tracked"))
def _bn_stats(x, running_mean, running_var, momentum, eps, updates, num_batches_tracked):
    return _K.bn_stats(x, running_mean, running_var, momentum, eps, updates, num_batches_tracked)


@_bn_stats.register_fake
def _(x, running_mean, running_var, momentum, eps, updates, num_batches_tracked):
    C = x.shape[1]
    return x.new_empty(C, dtype=torch.float32), x.new_empty(C, dtype=torch.float32)


def bn_stats(x2d, running_mean=None, running_var=None, momentum=0.1, eps=1e-5, updates=1, num_batches=None):
    return torch.ops.ssl_mae.bn_stats(x2d, running_mean, running_var, float(momentum), float(eps), int(updates),
                                      num_batches)


@_op("bn_eval_params", "(Tensor running_mean, Tensor running_var, float eps) -> (Tensor, Tensor)")
def _bn_eval_params(running_mean, running_var, eps):
    class _BN:
        pass
    bn = _BN()
    bn.running_mean, bn.running_var, bn.eps = running_mean, running_var, eps
    return _K.bn_eval_params(bn)


_bn_eval_params.register_fake(lambda rm, rv, eps: (torch.empty_like(rm), torch.empty_like(rm)))


def bn_eval_params(bn):
    return torch.ops.ssl_mae.bn_eval_params(bn.running_mean, bn.running_var, float(bn.eps))


@_op("bn_apply", "(Tensor x, Tensor mean, Tensor rstd, Tensor w, Tensor b, bool gelu, ScalarType? out_dtype, "
                 "Tensor? residual, Tensor? row_scale, int rows_per_group) -> Tensor")
def _bn_apply(x, mean, rstd, w, b, gelu, out_dtype, residual, row_scale, rows_per_group):
    return _K.bn_apply(x, mean, rstd, w, b, gelu, out_dtype, residual, row_scale, rows_per_group)


_bn_apply.register_fake(lambda x, mean, rstd, w, b, gelu, out_dtype, *a: x.new_empty(x.shape,
                                                                                     dtype=out_dtype or x.dtype))


def bn_apply(x2d, mean, rstd, w, b, gelu=False, out_dtype=None, residual=None, row_scale=None, rows_per_group=1,
             residual_bn=None):
    """residual_bn = (mean, rstd, weight, bias[, gelu False]): the residual is stored before
    its own BatchNorm (the stem's a2 under stages[0][0]) and enters as bf16(BN(residual))."""
    if residual_bn is not None:
        if len(residual_bn) > 4 and residual_bn[4]:
            raise ValueError("bn_apply: the residual's BatchNorm has no GELU")
        return torch.ops.ssl_mae.bn_apply_res_bn(x2d, mean, rstd, w, b, bool(gelu), out_dtype, residual,
                                                 *residual_bn[:4], row_scale, int(rows_per_group))
    return torch.ops.ssl_mae.bn_apply(x2d, mean, rstd, w, b, bool(gelu), out_dtype, residual, row_scale,
                                      int(rows_per_group))


@_op("bn_bwd", "(Tensor dy, Tensor x, Tensor mean, Tensor rstd, Tensor w, Tensor b, bool gelu, Tensor(a!) dw_sink, "
               "Tensor(b!) db_sink, Tensor? row_scale, int rows_per_group) -> Tensor", ("dw_sink", "db_sink"))
def _bn_bwd(dy, x, mean, rstd, w, b, gelu, dw_sink, db_sink, row_scale, rows_per_group):
    return _K.bn_bwd(dy, x, mean, rstd, w, b, gelu, dw_sink, db_sink, row_scale, rows_per_group)


_bn_bwd.register_fake(lambda dy, *a: torch.empty_like(dy))


def bn_bwd(dy, x2d, mean, rstd, w, b, gelu, dw_sink, db_sink, row_scale=None, rows_per_group=1):
    return torch.ops.ssl_mae.bn_bwd(dy, x2d, mean, rstd, w, b, bool(gelu), dw_sink, db_sink, row_scale,
                                    int(rows_per_group))


# ============================================================================ elementwise
@_op("gelu", "(Tensor x, float drop_p, int seed) -> Tensor")
def _gelu(x, drop_p, seed):
    return _K.gelu(x, drop_p, _u64(seed))


_gelu.register_fake(lambda x, p, s: torch.empty_like(x))


def _gelu_ctx(ctx, inputs, output):
    ctx.save_for_backward(inputs[0])
    ctx.args = inputs[1:]


def _gelu_bwd_formula(ctx, dy):
    (x,) = ctx.saved_tensors
    return gelu_bwd(x, dy.to(x.dtype).contiguous(), ctx.args[0], _u64(ctx.args[1])), None, None


_gelu.register_autograd(_gelu_bwd_formula, setup_context=_gelu_ctx)


def gelu(x, drop_p=0.0, seed=0):
    return torch.ops.ssl_mae.gelu(x, float(drop_p), _s64(seed))


@_op("gelu_bwd", "(Tensor pre, Tensor dy, float drop_p, int seed) -> Tensor")
def _gelu_bwd(pre, dy, drop_p, seed):
    return _K.gelu_bwd(pre, dy, drop_p, _u64(seed))


_gelu_bwd.register_fake(lambda pre, dy, p, s: torch.empty_like(dy))


def gelu_bwd(pre, dy, drop_p=0.0, seed=0):
    return torch.ops.ssl_mae.gelu_bwd(pre, dy, float(drop_p), _s64(seed))


@_op("dropout_bwd", "(Tensor dy, float drop_p, int seed, Tensor? row_scale, int rows_per_group) -> Tensor")
def _dropout_bwd(dy, drop_p, seed, row_scale, rows_per_group):
    return _K.dropout_bwd(dy, drop_p, _u64(seed), row_scale, rows_per_group)


_dropout_bwd.register_fake(lambda dy, *a: torch.empty_like(dy))


def dropout_bwd(dy, drop_p=0.0, seed=0, row_scale=None, rows_per_group=1):
    return torch.ops.ssl_mae.dropout_bwd(dy, float(drop_p), _s64(seed), row_scale, int(rows_per_group))


@_op("cast_dropout_bwd", "(Tensor dy, float drop_p, int seed, Tensor? row_scale, int rows_per_group) -> Tensor")
def _cast_dropout_bwd(dy, drop_p, seed, row_scale, rows_per_group):
    return _K.cast_dropout_bwd(dy, drop_p, _u64(seed), row_scale, rows_per_group)


_cast_dropout_bwd.register_fake(lambda dy, *a: torch.empty(dy.shape, dtype=torch.bfloat16, device=dy.device))


def cast_dropout_bwd(dy, drop_p=0.0, seed=0, row_scale=None, rows_per_group=1):
    return torch.ops.ssl_mae.cast_dropout_bwd(dy, float(drop_p), _s64(seed), row_scale, int(rows_per_group))


@_op("droppath_scale", "(int n, float p, int seed, Device device) -> Tensor")
def _droppath_scale(n, p, seed, device):
    return _K.droppath_scale(n, p, _u64(seed), device)


_droppath_scale.register_fake(lambda n, p, s, device: torch.empty(n, dtype=torch.float32, device=device))


def droppath_scale(n, p, seed, device):
    return torch.ops.ssl_mae.droppath_scale(int(n), float(p), _s64(seed), torch.device(device))


@_op("cast", "(Tensor a, ScalarType dtype) -> Tensor")
def _cast(a, dtype):
    return _K.cast(a, dtype)


_cast.register_fake(lambda a, dtype: a.new_empty(a.shape, dtype=dtype))


@_op("cast_into", "(Tensor a, Tensor(a!) out) -> ()", ("out",))
def _cast_into(a, out):
    _K.cast(a, out.dtype, out=out)


_cast_into.register_fake(_none)


def cast(a, dtype, out=None):
    if out is not None:
        torch.ops.ssl_mae.cast_into(a, out)
        return out
    return torch.ops.ssl_mae.cast(a, dtype)


@_op("fill_", "(Tensor(a!) t, float v) -> ()", ("t",))
def _fill(t, v):
    _K.fill_(t, v)


_fill.register_fake(_none)


def fill_(t, v):
    torch.ops.ssl_mae.fill_(t, float(v))
    return t


@_op("scale_", "(Tensor(a!) t, float a) -> ()", ("t",))
def _scale(t, a):
    _K.scale_(t, a)


_scale.register_fake(_none)


def scale_(t, a):
    torch.ops.ssl_mae.scale_(t, float(a))
    return t


# ============================================================================ convolutions
@_op("stem_im2col", "(Tensor clip, ScalarType out_dtype) -> Tensor")
def _stem_im2col(clip, out_dtype):
    return _K.stem_im2col(clip, out_dtype)[0]


@_stem_im2col.register_fake
def _(clip, out_dtype):
    if clip.dim() == 5:
        B, C, T, H, W = clip.shape
    else:
        B, C, H, W = clip.shape
        T = 1
    return clip.new_empty((B * T * ((H + 1) // 2) * ((W + 1) // 2), 32), dtype=out_dtype)


def stem_im2col(clip, out_dtype):
    if clip.dim() == 5:
        B, C, T, H, W = clip.shape
    else:
        B, C, H, W = clip.shape
        T = 1
    return torch.ops.ssl_mae.stem_im2col(clip, out_dtype), (B * T, (H + 1) // 2, (W + 1) // 2)


@_op("im2col3", "(Tensor x, int F, int H, int W, int C, int stride) -> Tensor")
def _im2col3(x, F, H, W, C, stride):
    return _K.im2col3(x, F, H, W, C, stride)


_im2col3.register_fake(lambda x, F, H, W, C, s: x.new_empty((F * ((H - 1) // s + 1) * ((W - 1) // s + 1), 9 * C)))


def im2col3(x, F, H, W, C, stride):
    return torch.ops.ssl_mae.im2col3(x, F, H, W, C, stride)


@_op("col2im3", "(Tensor dcol, int F, int H, int W, int C, int stride) -> Tensor")
def _col2im3(dcol, F, H, W, C, stride):
    return _K.col2im3(dcol, F, H, W, C, stride)


_col2im3.register_fake(lambda d, F, H, W, C, s: d.new_empty((F * H * W, C)))


def col2im3(dcol, F, H, W, C, stride):
    return torch.ops.ssl_mae.col2im3(dcol, F, H, W, C, stride)


@_op("conv_wpack", "(Tensor w, int Kpad, int order, ScalarType dtype) -> Tensor")
def _conv_wpack(w, Kpad, order, dtype):
    return _K.conv_wpack(w, Kpad, order, dtype)


_conv_wpack.register_fake(lambda w, Kpad, order, dtype: w.new_empty((w.shape[1] if order == 2 else w.shape[0], Kpad),
                                                                    dtype=dtype))


def conv_wpack(w, Kpad, order, dtype):
    return torch.ops.ssl_mae.conv_wpack(w, Kpad, order, dtype)


@_op("conv_wunpack_add", "(Tensor packed, Tensor(a!) grad, int order) -> ()", ("grad",))
def _conv_wunpack_add(packed, grad, order):
    _K.conv_wunpack_add(packed, grad, order)


_conv_wunpack_add.register_fake(_none)


def conv_wunpack_add(packed, grad, order):
    torch.ops.ssl_mae.conv_wunpack_add(packed, grad, order)


@_op("conv3x3_fwd", "(Tensor x, Tensor wpack, int F, int H, int W, int Cin, int Cout) -> Tensor")
def _conv3x3_fwd(x, wpack, F, H, W, Cin, Cout):
    return _K.conv3x3_fwd(x, wpack, F, H, W, Cin, Cout)


_conv3x3_fwd.register_fake(lambda x, w, F, H, W, Cin, Cout: x.new_empty((F * H * W, Cout)))


def conv3x3_fwd(x, wpack, F, H, W, Cin, Cout):
    return torch.ops.ssl_mae.conv3x3_fwd(x, wpack, F, H, W, Cin, Cout)


@_op("stem_conv1_bn_stats", "(Tensor clip, Tensor wpack, Tensor(a!)? running_mean, Tensor(b!)? running_var, "
                            "float momentum, float eps, int updates, Tensor(c!)? num_batches_tracked) "
                            "-> (Tensor, Tensor, Tensor)",
     ("running_mean", "running_var", "num_batches_tracked"))
def _stem_conv1_bn_stats(clip, wpack, running_mean, running_var, momentum, eps, updates, num_batches_tracked):
    return _K.stem_conv1_bn_stats(clip, wpack, running_mean, running_var, momentum, eps, updates,
                                  num_batches_tracked)[:3]


@_stem_conv1_bn_stats.register_fake
def _(clip, wpack, *a):
    if clip.dim() == 5:
        F, H, W = clip.shape[0] * clip.shape[2], clip.shape[3], clip.shape[4]
    else:
        F, H, W = clip.shape[0], clip.shape[2], clip.shape[3]
    P = F * ((H + 1) // 2) * ((W + 1) // 2)
    return (clip.new_empty((P, 48), dtype=torch.bfloat16), clip.new_empty(48, dtype=torch.float32),
            clip.new_empty(48, dtype=torch.float32))


def stem_conv1_bn_stats(clip, wpack, bn, updates=1):
    """Stem conv1 from the clip + the train-mode statistics of its BatchNorm (no im2col buffer).
    Returns (y, mean, rstd, (F, Ho, Wo))."""
    if clip.dim() == 5:
        F, H, W = clip.shape[0] * clip.shape[2], clip.shape[3], clip.shape[4]
    else:
        F, H, W = clip.shape[0], clip.shape[2], clip.shape[3]
    y, m, r = torch.ops.ssl_mae.stem_conv1_bn_stats(clip, wpack, bn.running_mean, bn.running_var,
                                                    float(bn.momentum), float(bn.eps), int(updates),
                                                    bn.num_batches_tracked)
    return y, m, r, (F, (H + 1) // 2, (W + 1) // 2)


@_op("stem_conv2_bn_stats", "(Tensor a1, Tensor bn1_mean, Tensor bn1_rstd, Tensor bn1_w, Tensor bn1_b, bool gelu, "
                            "Tensor wpack, int F, int H, int W, Tensor(a!)? running_mean, Tensor(b!)? running_var, "
                            "float momentum, float eps, int updates, Tensor(c!)? num_batches_tracked) "
                            "-> (Tensor, Tensor, Tensor)",
     ("running_mean", "running_var", "num_batches_tracked"))
def _stem_conv2_bn_stats(a1, m, r, g, b, gelu, wpack, F, H, W, running_mean, running_var, momentum, eps, updates,
                         num_batches_tracked):
    return _K.stem_conv2_bn_stats(a1, (m, r, g, b, gelu), wpack, F, H, W, running_mean, running_var, momentum, eps,
                                  updates, num_batches_tracked)


@_stem_conv2_bn_stats.register_fake
def _(a1, m, r, g, b, gelu, wpack, F, H, W, *a):
    return (a1.new_empty((F * H * W, 96), dtype=torch.bfloat16), a1.new_empty(96, dtype=torch.float32),
            a1.new_empty(96, dtype=torch.float32))


def stem_conv2_bn_stats(a1, act, wpack, F, H, W, bn, updates=1):
    """Stem conv2 over act(a1) (BN1 + GELU applied on the fly, h1 never written) + the
    train-mode statistics of BN2."""
    m, r, g, b, gelu = act
    return torch.ops.ssl_mae.stem_conv2_bn_stats(a1, m, r, g, b, bool(gelu), wpack, F, H, W, bn.running_mean,
                                                 bn.running_var, float(bn.momentum), float(bn.eps), int(updates),
                                                 bn.num_batches_tracked)


@_op("conv3x3_fwd_bn_stats", "(Tensor x, Tensor wpack, int F, int H, int W, int Cin, int Cout, "
                             "Tensor(a!)? running_mean, Tensor(b!)? running_var, float momentum, float eps, "
                             "int updates, Tensor(c!)? num_batches_tracked) -> (Tensor, Tensor, Tensor)",
     ("running_mean", "running_var", "num_batches_tracked"))
def _conv3x3_fwd_bn_stats(x, wpack, F, H, W, Cin, Cout, running_mean, running_var, momentum, eps, updates,
                          num_batches_tracked):
    return _K.conv3x3_fwd_bn_stats(x, wpack, F, H, W, Cin, Cout, running_mean, running_var, momentum, eps, updates,
                                   num_batches_tracked)


@_conv3x3_fwd_bn_stats.register_fake
def _(x, w, F, H, W, Cin, Cout, *a):
    return (x.new_empty((F * H * W, Cout), dtype=torch.bfloat16), x.new_empty(Cout, dtype=torch.float32),
            x.new_empty(Cout, dtype=torch.float32))


def conv3x3_fwd_bn_stats(x, wpack, F, H, W, Cin, Cout, bn, updates=1):
    """Stem conv2 + the train-mode statistics of its BatchNorm from the GEMM's epilogue."""
    return torch.ops.ssl_mae.conv3x3_fwd_bn_stats(x, wpack, F, H, W, Cin, Cout, bn.running_mean, bn.running_var,
                                                  float(bn.momentum), float(bn.eps), int(updates),
                                                  bn.num_batches_tracked)


@_op("conv3x3_dgrad", "(Tensor dy, Tensor wpack_t, int F, int H, int W, int Cin, int Cout) -> Tensor")
def _conv3x3_dgrad(dy, wpack_t, F, H, W, Cin, Cout):
    return _K.conv3x3_dgrad(dy, wpack_t, F, H, W, Cin, Cout)


_conv3x3_dgrad.register_fake(lambda dy, w, F, H, W, Cin, Cout: dy.new_empty((F * H * W, Cin)))


def conv3x3_dgrad(dy, wpack_t, F, H, W, Cin, Cout):
    return torch.ops.ssl_mae.conv3x3_dgrad(dy, wpack_t, F, H, W, Cin, Cout)


@_op("conv3x3_wgrad", "(Tensor dy, Tensor x, Tensor(a!) dw_sink, int F, int H, int W, int Cin, int Cout, "
                      "bool accumulate) -> ()", ("dw_sink",))
def _conv3x3_wgrad(dy, x, dw_sink, F, H, W, Cin, Cout, accumulate):
    _K.conv3x3_wgrad(dy, x, dw_sink, F, H, W, Cin, Cout, accumulate)


_conv3x3_wgrad.register_fake(_none)


def conv3x3_wgrad(dy, x, dw_sink, F, H, W, Cin, Cout, accumulate=True):
    torch.ops.ssl_mae.conv3x3_wgrad(dy, x, dw_sink, F, H, W, Cin, Cout, bool(accumulate))
    return dw_sink


@_op("dwconv", "(Tensor x, Tensor w, int F, int H, int W, int C, int stride) -> Tensor")
def _dwconv(x, w, F, H, W, C, stride):
    return _K.dwconv(x, w, F, H, W, C, stride)


_dwconv.register_fake(lambda x, w, F, H, W, C, s: x.new_empty((F * ((H - 1) // s + 1) * ((W - 1) // s + 1), C)))


def dwconv(x, w, F, H, W, C, stride):
    return torch.ops.ssl_mae.dwconv(x, w, F, H, W, C, stride)


@_op("dwconv_bwd", "(Tensor dy, Tensor x, Tensor w, Tensor(a!) dw_sink, int F, int H, int W, int C, int stride) "
                   "-> Tensor", ("dw_sink",))
def _dwconv_bwd(dy, x, w, dw_sink, F, H, W, C, stride):
    return _K.dwconv_bwd(dy, x, w, dw_sink, F, H, W, C, stride)


_dwconv_bwd.register_fake(lambda dy, x, *a: torch.empty_like(x))


def dwconv_bwd(dy, x, w, dw_sink, F, H, W, C, stride, need_dx=True):
    return torch.ops.ssl_mae.dwconv_bwd(dy, x, w, dw_sink, F, H, W, C, stride)


def _act(act):
    if act is None:
        return None, None, None, None, False
    m, r, w, b, g = act
    return m, r, w, b, bool(g)


@_op("dwconv_fused", "(Tensor x, Tensor? act_mean, Tensor? act_rstd, Tensor? act_w, Tensor? act_b, bool act_gelu, "
                     "Tensor w, int F, int H, int W, int C, int stride, bool with_stats, Tensor(a!)? running_mean, "
                     "Tensor(b!)? running_var, Tensor(c!)? num_batches_tracked, float momentum, float eps, "
                     "int updates) -> (Tensor, Tensor, Tensor)", ("running_mean", "running_var", "num_batches_tracked"))
def _dwconv_fused(x, am, ar, aw, ab, ag, w, F, H, W, C, stride, with_stats, rm, rv, nbt, momentum, eps, updates):
    act = None if am is None else (am, ar, aw, ab, ag)
    if not with_stats:
        return _K.dwconv_fused(x, act, w, F, H, W, C, stride), _e(x), _e(x)

    class _BN:
        pass
    bn = _BN()
    bn.running_mean, bn.running_var, bn.num_batches_tracked, bn.momentum, bn.eps = rm, rv, nbt, momentum, eps
    return _K.dwconv_fused(x, act, w, F, H, W, C, stride, bn_out=bn, bn_updates=updates)


@_dwconv_fused.register_fake
def _(x, am, ar, aw, ab, ag, w, F, H, W, C, stride, with_stats, *a):
    Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
    n = C if with_stats else 0
    return (x.new_empty((F * Ho * Wo, C)), x.new_empty(n, dtype=torch.float32),
            x.new_empty(n, dtype=torch.float32))


def dwconv_fused(x, act, w, F, H, W, C, stride, bn_out=None, bn_updates=1):
    if bn_out is None:
        return torch.ops.ssl_mae.dwconv_fused(x, *_act(act), w, F, H, W, C, stride, False, None, None, None, 0.1,
                                              1e-5, 1)[0]
    return torch.ops.ssl_mae.dwconv_fused(x, *_act(act), w, F, H, W, C, stride, True, bn_out.running_mean,
                                          bn_out.running_var, bn_out.num_batches_tracked, float(bn_out.momentum),
                                          float(bn_out.eps), int(bn_updates))


@_op("dwconv_fused_bwd", "(Tensor dy, Tensor x, Tensor? act_mean, Tensor? act_rstd, Tensor? act_w, Tensor? act_b, "
                         "bool act_gelu, Tensor w, Tensor(a!) dw_sink, int F, int H, int W, int C, int stride) -> Tensor",
     ("dw_sink",))
def _dwconv_fused_bwd(dy, x, am, ar, aw, ab, ag, w, dw_sink, F, H, W, C, stride):
    act = None if am is None else (am, ar, aw, ab, ag)
    return _K.dwconv_fused_bwd(dy, x, act, w, dw_sink, F, H, W, C, stride)


_dwconv_fused_bwd.register_fake(lambda dy, x, *a: torch.empty_like(x))


def dwconv_fused_bwd(dy, x, act, w, dw_sink, F, H, W, C, stride, need_dx=True):
    return torch.ops.ssl_mae.dwconv_fused_bwd(dy, x, *_act(act), w, dw_sink, F, H, W, C, stride)


@_op("dwconv_bn_bwd", "(Tensor dy, Tensor x, Tensor bn_mean, Tensor bn_rstd, Tensor bn_w, Tensor bn_b, "
                      "bool bn_gelu, Tensor w, Tensor(a!) dw_sink, Tensor(b!) dg_sink, Tensor(c!) db_sink, int F, "
                      "int H, int W, int C, int stride=1) -> Tensor", ("dw_sink", "dg_sink", "db_sink"))
def _dwconv_bn_bwd(dy, x, bm, br, bw, bb, bg, w, dw_sink, dg_sink, db_sink, F, H, W, C, stride=1):
    return _K.dwconv_bn_bwd(dy, x, (bm, br, bw, bb, bg), w, dw_sink, dg_sink, db_sink, F, H, W, C, stride)


_dwconv_bn_bwd.register_fake(lambda dy, x, *a: torch.empty_like(x))


def dwconv_bn_bwd(dy, x, act, w, dw_sink, dg_sink, db_sink, F, H, W, C, stride=1):
    return torch.ops.ssl_mae.dwconv_bn_bwd(dy, x, *_act(act), w, dw_sink, dg_sink, db_sink, F, H, W, C, int(stride))


# ============================================================================ SE
@_op("se_fwd", "(Tensor x, int F, int HW, int C, Tensor w1, Tensor w2, Tensor? act_mean, Tensor? act_rstd, "
               "Tensor? act_w, Tensor? act_b, bool act_gelu) -> (Tensor, Tensor, Tensor, Tensor)")
def _se_fwd(x, F, HW, C, w1, w2, am, ar, aw, ab, ag):
    act = None if am is None else (am, ar, aw, ab, ag)
    return _K.se_fwd(x, F, HW, C, w1, w2, act=act)


@_se_fwd.register_fake
def _(x, F, HW, C, w1, w2, *a):
    R = w1.shape[0]
    f = torch.float32
    return torch.empty_like(x), x.new_empty((F, C), dtype=f), x.new_empty((F, R), dtype=f), x.new_empty((F, C), dtype=f)


def se_fwd(x, F, HW, C, w1, w2, act=None):
    return torch.ops.ssl_mae.se_fwd(x, F, HW, C, w1, w2, *_act(act))


@_op("se_gate", "(Tensor x, int F, int HW, int C, Tensor w1, Tensor w2, Tensor? act_mean, Tensor? act_rstd, "
                "Tensor? act_w, Tensor? act_b, bool act_gelu) -> (Tensor, Tensor, Tensor)")
def _se_gate(x, F, HW, C, w1, w2, am, ar, aw, ab, ag):
    act = None if am is None else (am, ar, aw, ab, ag)
    return _K.se_fwd(x, F, HW, C, w1, w2, act=act, want_y=False)[1:]


@_se_gate.register_fake
def _(x, F, HW, C, w1, w2, *a):
    R = w1.shape[0]
    f = torch.float32
    return x.new_empty((F, C), dtype=f), x.new_empty((F, R), dtype=f), x.new_empty((F, C), dtype=f)


def se_gate(x, F, HW, C, w1, w2, act=None):
    """SELayer's pooled / hidden / gate without the scaled output (sm_se_fwd, y = null):
    the consumer forms act(x) * gate in its own loads (linear_se)."""
    return torch.ops.ssl_mae.se_gate(x, F, HW, C, w1, w2, *_act(act))


@_op("se_scale", "(Tensor x, Tensor s, int F, int HW, int C, Tensor? act_mean, Tensor? act_rstd, Tensor? act_w, "
                 "Tensor? act_b, bool act_gelu) -> Tensor")
def _se_scale(x, s, F, HW, C, am, ar, aw, ab, ag):
    act = None if am is None else (am, ar, aw, ab, ag)
    return _K.se_scale(x, s, F, HW, C, act=act)


_se_scale.register_fake(lambda x, *a: torch.empty_like(x))


def se_scale(x, s, F, HW, C, act=None):
    return torch.ops.ssl_mae.se_scale(x, s, F, HW, C, *_act(act))


@_op("linear_bn_stats", "(Tensor x, Tensor w, Tensor(a!)? running_mean, Tensor(b!)? running_var, float momentum, "
                        "float eps, int updates, Tensor(c!)? num_batches_tracked) -> (Tensor, Tensor, Tensor)",
     ("running_mean", "running_var", "num_batches_tracked"))
def _linear_bn_stats(x, w, running_mean, running_var, momentum, eps, updates, num_batches_tracked):
    return _K.linear_bn_stats(x, w, running_mean, running_var, momentum, eps, updates, num_batches_tracked)


@_linear_bn_stats.register_fake
def _(x, w, *a):
    N = w.shape[0]
    return (x.new_empty((x.shape[0], N), dtype=torch.bfloat16), x.new_empty(N, dtype=torch.float32),
            x.new_empty(N, dtype=torch.float32))


def linear_bn_stats(x, w, bn, updates=1):
    """Linear (1x1 conv) + the train-mode statistics of its BatchNorm from the GEMM's
    epilogue; bn = the BatchNorm2d module (running statistics updated `updates` times)."""
    return torch.ops.ssl_mae.linear_bn_stats(x, w, bn.running_mean, bn.running_var, float(bn.momentum),
                                             float(bn.eps), int(updates), bn.num_batches_tracked)


@_op("linear_bnin", "(Tensor a, Tensor a_mean, Tensor a_rstd, Tensor a_w, Tensor a_b, Tensor w) -> Tensor")
def _linear_bnin(a, am, ar, aw, ab, w):
    return _K.linear_bnin(a, (am, ar, aw, ab, False), w)


_linear_bnin.register_fake(lambda a, am, ar, aw, ab, w: a.new_empty((a.shape[0], w.shape[0]), dtype=torch.bfloat16))


@_op("linear_bnin_bn_stats", "(Tensor a, Tensor a_mean, Tensor a_rstd, Tensor a_w, Tensor a_b, Tensor w, "
                             "Tensor(a!)? running_mean, Tensor(b!)? running_var, float momentum, float eps, "
                             "int updates, Tensor(c!)? num_batches_tracked) -> (Tensor, Tensor, Tensor)",
     ("running_mean", "running_var", "num_batches_tracked"))
def _linear_bnin_bn_stats(a, am, ar, aw, ab, w, running_mean, running_var, momentum, eps, updates,
                          num_batches_tracked):
    return _K.linear_bnin(a, (am, ar, aw, ab, False), w,
                          (running_mean, running_var, momentum, eps, num_batches_tracked), updates)


@_linear_bnin_bn_stats.register_fake
def _(a, am, ar, aw, ab, w, *rest):
    N = w.shape[0]
    return (a.new_empty((a.shape[0], N), dtype=torch.bfloat16), a.new_empty(N, dtype=torch.float32),
            a.new_empty(N, dtype=torch.float32))


def linear_bnin(a, act, w, bn=None, updates=1):
    """Linear (1x1 conv) over the BatchNorm output x = bf16(BN(a)) formed in the GEMM's
    operand loads (act = (mean, rstd, weight, bias, False): the stem's BN2 feeding
    stages[0][0]); with bn (the consumer's BatchNorm2d module) also that BatchNorm's
    train-mode statistics from the epilogue (-> (y, mean, rstd))."""
    if act[4]:
        raise ValueError("linear_bnin: the folded BatchNorm has no GELU")
    if bn is None:
        return torch.ops.ssl_mae.linear_bnin(a, *act[:4], w)
    return torch.ops.ssl_mae.linear_bnin_bn_stats(a, *act[:4], w, bn.running_mean, bn.running_var,
                                                  float(bn.momentum), float(bn.eps), int(updates),
                                                  bn.num_batches_tracked)


@_op("bn_apply_res_bn", "(Tensor x, Tensor mean, Tensor rstd, Tensor w, Tensor b, bool gelu, ScalarType? out_dtype, "
                        "Tensor residual, Tensor r_mean, Tensor r_rstd, Tensor r_w, Tensor r_b, Tensor? row_scale, "
                        "int rows_per_group) -> Tensor")
def _bn_apply_res_bn(x, mean, rstd, w, b, gelu, out_dtype, residual, rm, rr, rw, rb, row_scale, rows_per_group):
    return _K.bn_apply(x, mean, rstd, w, b, gelu, out_dtype, residual, row_scale, rows_per_group,
                       residual_bn=(rm, rr, rw, rb))


_bn_apply_res_bn.register_fake(lambda x, mean, rstd, w, b, gelu, out_dtype, *a: x.new_empty(x.shape,
                                                                                           dtype=out_dtype or x.dtype))


@_op("linear_se", "(Tensor a2, Tensor w, Tensor act_mean, Tensor act_rstd, Tensor act_w, Tensor act_b, "
                  "bool act_gelu, Tensor gate, int hw) -> Tensor")
def _linear_se(a2, w, am, ar, aw, ab, ag, gate, hw):
    return _K.linear_se(a2, w, (am, ar, aw, ab, ag), gate, hw)


_linear_se.register_fake(lambda a2, w, *a: a2.new_empty((a2.shape[0], w.shape[0]), dtype=torch.bfloat16))


def linear_se(a2, w, act, gate, hw):
    """Forward of the MBConv projection over the SE output, h3 formed on load."""
    return torch.ops.ssl_mae.linear_se(a2, w, *act[:4], bool(act[4]), gate, int(hw))


@_op("linear_dw_se", "(Tensor dy, Tensor a2, Tensor act_mean, Tensor act_rstd, Tensor act_w, Tensor act_b, "
                     "bool act_gelu, Tensor? gate, int hw, Tensor(a!) grad_sink, bool accumulate) -> ()", ("grad_sink",))
def _linear_dw_se(dy, a2, am, ar, aw, ab, ag, gate, hw, grad_sink, accumulate):
    _K.linear_dw_se(dy, a2, (am, ar, aw, ab, ag), gate, hw, grad_sink, accumulate)


_linear_dw_se.register_fake(_none)


def linear_dw_se(dy, a2, act, gate, hw, grad_sink, accumulate=True):
    """Weight gradient of the MBConv projection over the SE output, h3 formed on load."""
    torch.ops.ssl_mae.linear_dw_se(dy, a2, *act[:4], bool(act[4]), gate, int(hw), grad_sink, bool(accumulate))
    return grad_sink


@_op("se_bwd", "(Tensor dy, Tensor x, int F, int HW, int C, Tensor w1, Tensor w2, Tensor s, Tensor h1, "
               "Tensor? act_mean, Tensor? act_rstd, Tensor? act_w, Tensor? act_b, bool act_gelu) "
               "-> (Tensor, Tensor, Tensor)")
def _se_bwd(dy, x, F, HW, C, w1, w2, s, h1, am, ar, aw, ab, ag):
    act = None if am is None else (am, ar, aw, ab, ag)
    return _K.se_bwd(dy, x, F, HW, C, w1, w2, s, h1, act=act)


@_se_bwd.register_fake
def _(dy, x, F, HW, C, w1, w2, *a):
    R = w1.shape[0]
    return torch.empty_like(x), x.new_empty((F, C), dtype=torch.float32), x.new_empty((F, R), dtype=torch.float32)


def se_bwd(dy, x, F, HW, C, w1, w2, s, h1, act=None):
    return torch.ops.ssl_mae.se_bwd(dy, x, F, HW, C, w1, w2, s, h1, *_act(act))


@_op("se_bn_bwd", "(Tensor dy, Tensor x, int F, int HW, int C, Tensor w1, Tensor w2, Tensor s, Tensor h1, "
                  "Tensor act_mean, Tensor act_rstd, Tensor act_w, Tensor act_b, bool act_gelu, Tensor(a!) dw_sink, "
                  "Tensor(b!) db_sink) -> (Tensor, Tensor, Tensor)", ("dw_sink", "db_sink"))
def _se_bn_bwd(dy, x, F, HW, C, w1, w2, s, h1, am, ar, aw, ab, ag, dw_sink, db_sink):
    return _K.se_bn_bwd(dy, x, F, HW, C, w1, w2, s, h1, (am, ar, aw, ab, ag), dw_sink, db_sink)


@_se_bn_bwd.register_fake
def _(dy, x, F, HW, C, w1, w2, *a):
    R = w1.shape[0]
    return torch.empty_like(x), x.new_empty((F, C), dtype=torch.float32), x.new_empty((F, R), dtype=torch.float32)


def se_bn_bwd(dy, x, F, HW, C, w1, w2, s, h1, act, dw_sink, db_sink):
    return torch.ops.ssl_mae.se_bn_bwd(dy, x, F, HW, C, w1, w2, s, h1, *_act(act), dw_sink, db_sink)


# ============================================================================ MAE glue
@_op("tube_mask", "(Tensor noise, int T, int n_mask) -> (Tensor, Tensor)")
def _tube_mask(noise, T, n_mask):
    return _K.tube_mask(noise, T, n_mask)


@_tube_mask.register_fake
def _(noise, T, n_mask):
    B, L = noise.shape
    return noise.new_empty((B, T, L), dtype=torch.uint8), noise.new_empty(B * T * n_mask, dtype=torch.int32)


def tube_mask(noise, T, n_mask, with_index=True):
    return torch.ops.ssl_mae.tube_mask(noise, T, n_mask)


@_op("pos_blend", "(Tensor y, Tensor tpos, Tensor spos, Tensor tok, Tensor mask, int B, int T, int L, int D, "
                  "ScalarType out_dtype) -> Tensor")
def _pos_blend(y, tpos, spos, tok, mask, B, T, L, D, out_dtype):
    return _K.pos_blend(y, tpos, spos, tok, mask, B, T, L, D, out_dtype)


_pos_blend.register_fake(lambda y, tp, sp, tok, m, B, T, L, D, dt: y.new_empty((B * T * L, D), dtype=dt))


def pos_blend(y, tpos, spos, tok, mask_u8, B, T, L, D, out_dtype):
    return torch.ops.ssl_mae.pos_blend(y, tpos, spos, tok, mask_u8, B, T, L, D, out_dtype)


@_op("pos_blend_bwd", "(Tensor dx, Tensor mask, ScalarType y_dtype, Tensor(a!) dtpos, Tensor(b!) dspos, "
                      "Tensor(c!) dtok, int B, int T, int L, int D) -> Tensor", ("dtpos", "dspos", "dtok"))
def _pos_blend_bwd(dx, mask, y_dtype, dtpos, dspos, dtok, B, T, L, D):
    return _K.pos_blend_bwd(dx, mask, y_dtype, dtpos, dspos, dtok, B, T, L, D)


_pos_blend_bwd.register_fake(lambda dx, m, ydt, *a: dx.new_empty(dx.shape, dtype=ydt))


def pos_blend_bwd(dx, mask_u8, y_dtype, dtpos, dspos, dtok, B, T, L, D):
    return torch.ops.ssl_mae.pos_blend_bwd(dx, mask_u8, y_dtype, dtpos, dspos, dtok, B, T, L, D)


@_op("mae_loss_fwd", "(Tensor pred, Tensor clip, Tensor mask, bool norm_pix) -> (Tensor, Tensor)")
def _mae_loss_fwd(pred, clip, mask, norm_pix):
    return _K.mae_loss_fwd(pred, clip, mask, norm_pix)


_mae_loss_fwd.register_fake(lambda pred, clip, mask, n: (pred.new_empty((), dtype=torch.float32),
                                                         pred.new_empty(1, dtype=torch.float32)))


def _loss_ctx(ctx, inputs, output):
    pred, clip, mask, norm_pix = inputs
    ctx.norm_pix = norm_pix
    ctx.save_for_backward(pred, clip, mask, output[1])


def _loss_bwd_formula(ctx, g, gdenom):
    pred, clip, mask, denom = ctx.saved_tensors
    return mae_loss_bwd(pred, clip, mask, ctx.norm_pix, g, denom), None, None, None


_mae_loss_fwd.register_autograd(_loss_bwd_formula, setup_context=_loss_ctx)


def mae_loss_fwd(pred, clip, mask_u8, norm_pix=True):
    return torch.ops.ssl_mae.mae_loss_fwd(pred, clip, mask_u8, bool(norm_pix))


@_op("mae_loss_bwd", "(Tensor pred, Tensor clip, Tensor mask, bool norm_pix, Tensor grad_out, Tensor denom) -> Tensor")
def _mae_loss_bwd(pred, clip, mask, norm_pix, grad_out, denom):
    return _K.mae_loss_bwd(pred, clip, mask, norm_pix, grad_out, denom)


_mae_loss_bwd.register_fake(lambda pred, *a: torch.empty_like(pred))


def mae_loss_bwd(pred, clip, mask_u8, norm_pix, grad_out, denom):
    return torch.ops.ssl_mae.mae_loss_bwd(pred, clip, mask_u8, bool(norm_pix), grad_out, denom)


@_op("patchify", "(Tensor imgs, int p) -> Tensor")
def _patchify(imgs, p):
    return _K.patchify(imgs, p)


@_patchify.register_fake
def _(imgs, p):
    B, C, T, H, W = imgs.shape
    return imgs.new_empty((B, T * (H // p) * (W // p), p * p * C), dtype=torch.float32)


def _patchify_ctx(ctx, inputs, output):
    ctx.shape = tuple(inputs[0].shape)
    ctx.p = inputs[1]


_patchify.register_autograd(lambda ctx, g: (unpatchify(g, *ctx.shape[1:], p=ctx.p), None),
                            setup_context=_patchify_ctx)


def patchify(imgs, p=8):
    return torch.ops.ssl_mae.patchify(imgs, p)


@_op("unpatchify", "(Tensor tokens, int C, int T, int H, int W, int p) -> Tensor")
def _unpatchify(tokens, C, T, H, W, p):
    return _K.unpatchify(tokens, C, T, H, W, p)


_unpatchify.register_fake(lambda t, C, T, H, W, p: t.new_empty((t.shape[0], C, T, H, W), dtype=torch.float32))


def unpatchify(tokens, C, T, H, W, p=8):
    return torch.ops.ssl_mae.unpatchify(tokens, C, T, H, W, p)


@_op("gather_rows", "(Tensor src, Tensor idx) -> Tensor")
def _gather_rows(src, idx):
    return _K.gather_rows(src, idx)


_gather_rows.register_fake(lambda src, idx: src.new_empty((idx.numel(), src.shape[1])))


def gather_rows(src2d, idx):
    return torch.ops.ssl_mae.gather_rows(src2d, idx)


@_op("std", "(Tensor x) -> Tensor")
def _std(x):
    return _K.std(x)


_std.register_fake(lambda x: x.new_empty((), dtype=torch.float32))


def std(x):
    return torch.ops.ssl_mae.std(x)


@_op("segment_mean", "(Tensor x, int G, int R, int C) -> Tensor")
def _segment_mean(x, G, R, C):
    return _K.segment_mean(x, G, R, C)


_segment_mean.register_fake(lambda x, G, R, C: x.new_empty((G, C), dtype=torch.float32))


def _segmean_ctx(ctx, inputs, output):
    ctx.args = (inputs[1], inputs[2], inputs[3], inputs[0].dtype)


_segment_mean.register_autograd(
    lambda ctx, g: (segment_mean_bwd(g.float().contiguous(), *ctx.args), None, None, None),
    setup_context=_segmean_ctx)


def segment_mean(x, G, R, C):
    return torch.ops.ssl_mae.segment_mean(x, G, R, C)


@_op("segment_mean_bwd", "(Tensor dy, int G, int R, int C, ScalarType dtype) -> Tensor")
def _segment_mean_bwd(dy, G, R, C, dtype):
    return _K.segment_mean_bwd(dy, G, R, C, dtype)


_segment_mean_bwd.register_fake(lambda dy, G, R, C, dtype: dy.new_empty((G * R, C), dtype=dtype))


def segment_mean_bwd(dy, G, R, C, dtype):
    return torch.ops.ssl_mae.segment_mean_bwd(dy, G, R, C, dtype)


# ============================================================================ optimizer
@_op("nonfinite", "(Tensor g, Tensor(a!) flag) -> ()", ("flag",))
def _nonfinite(g, flag):
    _K.nonfinite(g, flag)


_nonfinite.register_fake(_none)


def nonfinite(g, flag):
    torch.ops.ssl_mae.nonfinite(g, flag)


@_op("adamw", "(Tensor(a!) p, Tensor g, Tensor(b!) m, Tensor(c!) v, float lr, float b1, float b2, float eps, "
              "float wd, Tensor found_inf, Tensor(d!) step, Tensor(e!)? shadow, bool advance_step) -> ()",
     ("p", "m", "v", "step", "shadow"))
def _adamw(p, g, m, v, lr, b1, b2, eps, wd, found_inf, step, shadow, advance_step):
    _K.adamw(p, g, m, v, lr, b1, b2, eps, wd, found_inf, step, shadow, advance_step)


_adamw.register_fake(_none)


def adamw(p, g, m, v, lr, b1, b2, eps, wd, found_inf, step, shadow=None, advance_step=True):
    torch.ops.ssl_mae.adamw(p, g, m, v, float(lr), float(b1), float(b2), float(eps), float(wd), found_inf, step,
                            shadow, bool(advance_step))


# ============================================================================ FedAvg / clip pipeline
@_op("fedavg_weighted_sum", "(Tensor[] bufs, float[] weights) -> Tensor")
def _fedavg_weighted_sum(bufs, weights):
    return _K.fedavg_weighted_sum(list(bufs), list(weights))


_fedavg_weighted_sum.register_fake(lambda bufs, w: torch.empty_like(bufs[0]))


def fedavg_weighted_sum(bufs, weights):
    return torch.ops.ssl_mae.fedavg_weighted_sum(list(bufs), [float(w) for w in weights])


@_op("fedavg_counters_max", "(Tensor[] bufs) -> Tensor")
def _fedavg_counters_max(bufs):
    return _K.fedavg_counters_max(list(bufs))


_fedavg_counters_max.register_fake(lambda bufs: torch.empty_like(bufs[0]))


def fedavg_counters_max(bufs):
    return torch.ops.ssl_mae.fedavg_counters_max(list(bufs))


@_op("frames_normalize", "(Tensor frames, float[] mean, float[] std, bool bgr_swap, Tensor? valid) -> Tensor")
def _frames_normalize(frames, mean, std, bgr_swap, valid):
    return _K.frames_normalize(frames, mean, std, bgr_swap, valid)


@_frames_normalize.register_fake
def _(frames, mean, std, bgr_swap, valid):
    B, T, H, W, _ = frames.shape
    return frames.new_empty((B, 3, T, H, W), dtype=torch.float32)


def frames_normalize(frames, mean, std, bgr_swap=True, valid=None):
    return torch.ops.ssl_mae.frames_normalize(frames, [float(x) for x in mean], [float(x) for x in std],
                                              bool(bgr_swap), valid)


def registered_ops():
    """Names of every ssl_mae operator registered by this module."""
    return sorted(n for n in dir(torch.ops.ssl_mae) if not n.startswith("_") and
                  isinstance(getattr(torch.ops.ssl_mae, n), torch._ops.OpOverloadPacket))
