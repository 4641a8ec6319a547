"""Autograd Functions of the MAE step: each one drives a fused group of HIP kernels
forward and backward (the "engine" of this framework).

Activations are token-major (channels-last): [rows][C].  Each Function saves
only what its backward cannot cheaply recompute (pre-BN conv outputs, attention
inputs/outputs, the GELU pre-activation) and recomputes BN/GELU/LN outputs in the
backward; everything saved goes through ctx.save_for_backward so that
torch.utils.checkpoint (the reference's per-stage checkpointing,
tiny_vit.py:170-173) can drop and replay it.  Weight gradients are written by the
kernels straight into the flat fp32 gradient buffer (optim.FlatParams); the
Functions return None for every parameter.

Precision policy (mirrors the reference under torch.autocast(bf16),
SURVEY.md §3.2): bf16 mode = bf16 activations/GEMM operands, fp32 accumulation,
LayerNorm/BN statistics in fp32, fp32 decoder residual stream with the branch
rounded to bf16 before the add, bf16 pred, fp32 loss.  fp32 mode = everything
fp32 (what the reference computes on a CPU-only host) — used for parity.
"""
import math

import torch

from . import ops as K    # every kernel launch through the torch.ops.ssl_mae dispatcher


class Mode:
    """Per-forward execution mode: precision and the base of the counter-hash RNG
    (dropout / DropPath masks are a pure function of (seed, element index), so the
    checkpoint recompute and the backward regenerate exactly the forward's masks)."""
    __slots__ = ("bf16", "act", "seed_base")

    def __init__(self, bf16, seed_base=0):
        self.bf16 = bool(bf16)
        self.act = torch.bfloat16 if bf16 else torch.float32
        self.seed_base = int(seed_base)

    def seed(self, module_index, site):
        return splitmix64(self.seed_base ^ splitmix64((module_index << 8) | site))


_M64 = (1 << 64) - 1


def splitmix64(x):
    x = (x + 0x9E3779B97F4A7C15) & _M64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & _M64
    return x ^ (x >> 31)


def W(p, mode):
    """GEMM operand view of a weight: bf16 shadow or the fp32 master."""
    return p._sm_bf16 if mode.bf16 else p.detach()


def G(p):
    return p._sm_grad


def _touch(*params):
    flat = getattr(params[0], "_sm_flat", None)
    if flat is None:
        raise RuntimeError("parameters are not registered in a FlatParams buffer")
    flat.touch(*params)


def _done(*params):
    """End of a backward kernel group: its gradient writes are enqueued, so the
    data-parallel bucket(s) holding these parameters may start reducing."""
    params[0]._sm_flat.done(*params)


def _bn_params(a2d, bn, updates=1):
    """(mean, rstd) of a BatchNorm2d: batch statistics in train mode (running stats
    updated `updates` times), the running statistics in eval mode."""
    if not bn.training:
        return K.bn_eval_params(bn)
    return K.bn_stats(a2d, bn.running_mean, bn.running_var, bn.momentum, bn.eps, updates, bn.num_batches_tracked)


def _bn_forward(a2d, bn, gelu, residual=None, updates=1):
    mean, rstd = _bn_params(a2d, bn, updates)
    y = K.bn_apply(a2d, mean, rstd, bn.weight.detach(), bn.bias.detach(), gelu=gelu, residual=residual)
    return y, mean, rstd


def _train_bn_only(ctx, *bns):
    """The fused backward kernels differentiate through batch statistics; the
    reference never backpropagates through eval-mode BatchNorm (train_finetune.py
    trains under model.train() and evaluates under no_grad)."""
    if not all(bn.training for bn in bns):
        raise NotImplementedError("backward through eval-mode BatchNorm is not supported (train-mode BN only)")


# ============================================================================ stem
class StemFn(torch.autograd.Function):
    """PatchEmbed (tiny_vit.py:62-72): conv3x3 s2 3->48, BN, GELU, conv3x3 s1 48->96, BN.
    Input: the clip [B,3,T,H,W] (or frames [N,3,H,W]); the frame permute of
    mae_vit_adapter.py:84 is folded into the im2col loads.

    Outputs (t, m2, r2).  With st.fold_bn2 (bf16 training, direct conv2 path) BN2's apply
    is folded into stages[0][0], its only consumer: t holds the conv2 output a2, NOT y =
    BN2(a2), and (m2, r2) are BN2's batch statistics; the consumer (MBConvFn with
    st.x_bn) forms y = bf16(a2 sc + sh) in its own loads exactly as bn_apply stores it
    and returns dL/dy as t's gradient, so y never exists in HBM.  Otherwise t = y and
    (m2, r2) are returned for reference only."""

    @staticmethod
    def forward(ctx, clip, st, w1, g1, b1, w2, g2, b2):
        mode = st.mode
        act = mode.act
        w1p = K.conv_wpack(w1.detach(), 32, 0, act)
        w2p = K.conv_wpack(w2.detach(), 432, 1, act)
        h1 = None
        if mode.bf16 and st.bn1.training:   # conv1 straight from the clip + BN1 statistics
            a1, m1, r1, (Fr, Ho, Wo) = K.stem_conv1_bn_stats(clip, w1p, st.bn1)
            if st.bn2.training and Wo <= 128:
                # conv2 over GELU(BN1(a1)) formed in its LDS ring (h1 never written) + BN2
                # statistics
                a2, m2, r2 = K.stem_conv2_bn_stats(a1, (m1, r1, g1.detach(), b1.detach(), True), w2p, Fr, Ho, Wo,
                                                   st.bn2)
                y = a2 if st.fold_bn2 else K.bn_apply(a2, m2, r2, g2.detach(), b2.detach(), gelu=False)
                ctx.folded = st.fold_bn2
            else:
                h1 = K.bn_apply(a1, m1, r1, g1.detach(), b1.detach(), gelu=True)
        else:
            col1, (Fr, Ho, Wo) = K.stem_im2col(clip, act)
            a1 = K.linear(col1, w1p)
            del col1
            h1, m1, r1 = _bn_forward(a1, st.bn1, gelu=True)
        if h1 is None:
            pass
        elif mode.bf16 and st.bn2.training:   # conv2 as a GEMM over the implicit im2col of h1
            # (no 9x buffer) with BN2's statistics from its epilogue (no read pass of a2)
            a2, m2, r2 = K.conv3x3_fwd_bn_stats(h1, w2p, Fr, Ho, Wo, 48, 96, st.bn2)
            del h1
            y = K.bn_apply(a2, m2, r2, g2.detach(), b2.detach(), gelu=False)
        else:
            if mode.bf16:
                a2 = K.conv3x3_fwd(h1, w2p, Fr, Ho, Wo, 48, 96)
            else:           # fp32 parity path: explicit im2col + exact-fp32 GEMM
                col2 = K.im2col3(h1, Fr, Ho, Wo, 48, 1)
                a2 = K.linear(col2, w2p)
                del col2
            del h1
            y, m2, r2 = _bn_forward(a2, st.bn2, gelu=False)
        if not getattr(ctx, "folded", False):
            ctx.folded = False
        ctx.st = st
        ctx.geom = (Fr, Ho, Wo)
        ctx.params = (w1, g1, b1, w2, g2, b2)
        ctx.save_for_backward(clip, a1, a2, m1, r1, m2, r2, w1p, w2p)
        ctx.mark_non_differentiable(m2, r2)
        return y.view(Fr, Ho, Wo, 96), m2, r2

    @staticmethod
    def backward(ctx, dy, _dm2=None, _dr2=None):
        _train_bn_only(ctx, ctx.st.bn1, ctx.st.bn2)
        clip, a1, a2, m1, r1, m2, r2, w1p, w2p = ctx.saved_tensors
        w1, g1, b1, w2, g2, b2 = ctx.params
        act = ctx.st.mode.act
        Fr, Ho, Wo = ctx.geom
        _touch(w1, g1, b1, w2, g2, b2)
        dy = dy.reshape(-1, 96).to(act).contiguous()
        da2 = K.bn_bwd(dy, a2, m2, r2, g2.detach(), b2.detach(), False, G(g2), G(b2))
        del dy
        h1 = K.bn_apply(a1, m1, r1, g1.detach(), b1.detach(), gelu=True)
        dw2p = torch.empty((96, 432), dtype=torch.float32, device=a1.device)
        if ctx.st.mode.bf16:     # implicit-im2col weight and data gradients
            K.conv3x3_wgrad(da2, h1, dw2p, Fr, Ho, Wo, 48, 96, accumulate=False)
            del h1
            dh1 = K.conv3x3_dgrad(da2, K.conv_wpack(w2.detach(), 864, 2, act), Fr, Ho, Wo, 48, 96)
            del da2
        else:
            col2 = K.im2col3(h1, Fr, Ho, Wo, 48, 1)
            del h1
            K.linear_dw(da2, col2, dw2p, accumulate=False)
            del col2
            dcol2 = K.linear_dx(da2, w2p)
            del da2
            dh1 = K.col2im3(dcol2, Fr, Ho, Wo, 48, 1)
            del dcol2
        K.conv_wunpack_add(dw2p, G(w2), 1)
        da1 = K.bn_bwd(dh1, a1, m1, r1, g1.detach(), b1.detach(), True, G(g1), G(b1))
        del dh1
        col1, _ = K.stem_im2col(clip, act)
        dw1p = torch.empty((48, 32), dtype=torch.float32, device=a1.device)
        K.linear_dw(da1, col1, dw1p, accumulate=False)
        K.conv_wunpack_add(dw1p, G(w1), 0)
        _done(*ctx.params)
        return (None,) * 8


# ============================================================================ MBConv
class MBConvFn(torch.autograd.Function):
    """MBConv + SELayer (tiny_vit.py:36-56, 20-34): 1x1 expand, BN, GELU, dw3x3
    (stride s), BN, GELU, SE, 1x1 project, BN (+ residual when s == 1, Cin == Cout).
    st.bn_updates: how many times the BatchNorm running statistics take this batch
    (2 reproduces a checkpointed stage's forward + recompute, TinyViT._run_stages);
    st.recompute_a1: drop the expand output a1 (the block's largest tensor) and
    recompute its GEMM in the backward (bit-identical: same kernel, same inputs);
    st.recompute_a2: also drop the depthwise output a2 and recompute it in the
    backward from a1 with the saved BN0 statistics (no running-stat update) -- the
    stage-0 "lite-resident" mode: two recomputed kernels instead of the whole
    checkpointed stage forward.
    st.x_bn = (mean, rstd, weight, bias): the input is stored before its BatchNorm (the
    stem's conv2 output under StemFn's folded BN2): every read of x -- the expand conv's
    A operand, the residual, the expand weight gradient's B operand -- forms bf16(BN(x))
    in its loads, bit-identical to reading the stored BN output."""

    @staticmethod
    def forward(ctx, x, st, w_exp, g0, b0, w_dw, g2, b2, w_fc0, w_fc2, w_proj, g5, b5):
        mode = st.mode
        Fr, H, Wd, Cin = x.shape
        mid, Cout, s = st.mid, st.cout, st.stride
        x2d = x.reshape(-1, Cin)
        Ho, Wo = (H - 1) // s + 1, (Wd - 1) // s + 1
        fused = mode.bf16 and mid % 32 == 0
        xbn = getattr(st, "x_bn", None)
        if xbn is not None:            # x = bf16(BN(stored)) formed in the expand GEMM's loads
            if not fused:
                raise NotImplementedError("a BatchNorm-folded input needs the fused bf16 MBConv")
            xbn = tuple(xbn[:4]) + (False,)
            if st.bn0.training:
                a1, m0, r0 = K.linear_bnin(x2d, xbn, W(w_exp, mode).view(mid, Cin), st.bn0, st.bn_updates)
            else:
                a1 = K.linear_bnin(x2d, xbn, W(w_exp, mode).view(mid, Cin))
        elif fused and st.bn0.training:   # expand conv + BN0 statistics from its epilogue
            a1, m0, r0 = K.linear_bn_stats(x2d, W(w_exp, mode).view(mid, Cin), st.bn0, st.bn_updates)
        else:
            a1 = K.linear(x2d, W(w_exp, mode).view(mid, Cin))
        if fused:
            # BN0 + GELU folded into the depthwise conv's loads, BN2 statistics produced
            # by it, BN2 + GELU folded into the SE reads: no act(a1) / act(a2) in HBM
            if not st.bn0.training:
                m0, r0 = _bn_params(a1, st.bn0, st.bn_updates)
            act0 = (m0, r0, g0.detach(), b0.detach(), True)
            if st.bn2.training:
                a2, m2, r2 = K.dwconv_fused(a1, act0, w_dw.detach().view(mid, 9), Fr, H, Wd, mid, s,
                                            bn_out=st.bn2, bn_updates=st.bn_updates)
            else:
                a2 = K.dwconv_fused(a1, act0, w_dw.detach().view(mid, 9), Fr, H, Wd, mid, s)
                m2, r2 = K.bn_eval_params(st.bn2)
            act2 = (m2, r2, g2.detach(), b2.detach(), True)
            if (Ho * Wo) % 128 == 0 and mid % 64 == 0 and mid <= 1536 and Cout <= 128:
                # SE gate only; the projection GEMM forms h3 = act(a2) * gate in its operand
                # loads (no h3 round trip; bit-identical to se_fwd's h3 + linear)
                pooled, h1se, gate = K.se_gate(a2, Fr, Ho * Wo, mid, w_fc0.detach(), w_fc2.detach(), act=act2)
                h3 = None
            else:
                h3, pooled, h1se, gate = K.se_fwd(a2, Fr, Ho * Wo, mid, w_fc0.detach(), w_fc2.detach(), act=act2)
        else:
            h1, m0, r0 = _bn_forward(a1, st.bn0, gelu=True, updates=st.bn_updates)
            a2 = K.dwconv(h1, w_dw.detach().view(mid, 9), Fr, H, Wd, mid, s)
            del h1
            h2, m2, r2 = _bn_forward(a2, st.bn2, gelu=True, updates=st.bn_updates)
            h3, pooled, h1se, gate = K.se_fwd(h2, Fr, Ho * Wo, mid, w_fc0.detach(), w_fc2.detach())
            del h2
        if h3 is None:
            a3 = K.linear_se(a2.view(-1, mid), W(w_proj, mode).view(Cout, mid), act2, gate, Ho * Wo)
        else:
            a3 = K.linear(h3, W(w_proj, mode).view(Cout, mid))
        del h3
        mean5, rstd5 = _bn_params(a3, st.bn5, st.bn_updates)
        out = K.bn_apply(a3, mean5, rstd5, g5.detach(), b5.detach(), residual=x2d if st.res else None,
                         row_scale=st.dp_scale, rows_per_group=Ho * Wo,
                         residual_bn=xbn if (st.res and xbn is not None) else None)
        m5, r5 = mean5, rstd5
        ctx.fused = fused
        ctx.xbn = xbn
        ctx.st = st
        ctx.geom = (Fr, H, Wd, Cin, Ho, Wo)
        ctx.params = (w_exp, g0, b0, w_dw, g2, b2, w_fc0, w_fc2, w_proj, g5, b5)
        lite = getattr(st, "recompute_a2", False)
        ctx.save_for_backward(x, None if (st.recompute_a1 or lite) else a1, None if lite else a2, a3, m0, r0, m2, r2,
                              m5, r5, pooled, h1se, gate)
        return out.view(Fr, Ho, Wo, Cout)

    @staticmethod
    def backward(ctx, dout):
        _train_bn_only(ctx, ctx.st.bn0, ctx.st.bn2, ctx.st.bn5)
        x, a1, a2, a3, m0, r0, m2, r2, m5, r5, pooled, h1se, gate = ctx.saved_tensors
        w_exp, g0, b0, w_dw, g2, b2, w_fc0, w_fc2, w_proj, g5, b5 = ctx.params
        st = ctx.st
        mode = st.mode
        Fr, H, Wd, Cin, Ho, Wo = ctx.geom
        mid, Cout, s = st.mid, st.cout, st.stride
        _touch(*ctx.params)
        xbn = ctx.xbn

        def expand(xin):        # recompute a1 = x W^T (same kernel form as the forward's)
            if xbn is not None:
                return K.linear_bnin(xin.reshape(-1, Cin), xbn, W(w_exp, mode).view(mid, Cin))
            return K.linear(xin.reshape(-1, Cin), W(w_exp, mode).view(mid, Cin))
        if a2 is None:          # lite-resident: a1 and a2 recomputed from x (same kernels, saved stats)
            a1 = expand(x)
            if ctx.fused:
                a2 = K.dwconv_fused(a1, (m0, r0, g0.detach(), b0.detach(), True), w_dw.detach().view(mid, 9), Fr,
                                    H, Wd, mid, s)
            else:
                a2 = K.dwconv(K.bn_apply(a1, m0, r0, g0.detach(), b0.detach(), gelu=True),
                              w_dw.detach().view(mid, 9), Fr, H, Wd, mid, s)
        dout2d = dout.reshape(-1, Cout).to(mode.act).contiguous()
        da3 = K.bn_bwd(dout2d, a3, m5, r5, g5.detach(), b5.detach(), False, G(g5), G(b5),
                       row_scale=st.dp_scale, rows_per_group=Ho * Wo)
        if ctx.fused:
            act2 = (m2, r2, g2.detach(), b2.detach(), True)
            if (Ho * Wo) % 64 == 0:
                # projection weight gradient with the SE output h3 formed in the GEMM's
                # operand loads (no h3 round trip; bit-identical to se_scale + linear_dw)
                K.linear_dw_se(da3, a2.view(-1, mid), act2, gate, Ho * Wo, G(w_proj).view(Cout, mid))
            else:
                h3 = K.se_scale(a2, gate, Fr, Ho * Wo, mid, act=act2)
                K.linear_dw(da3, h3, G(w_proj).view(Cout, mid))
                del h3
        else:
            h2 = K.bn_apply(a2, m2, r2, g2.detach(), b2.detach(), gelu=True)
            h3 = K.se_scale(h2, gate, Fr, Ho * Wo, mid)
            K.linear_dw(da3, h3, G(w_proj).view(Cout, mid))
            del h3
        dh3 = K.linear_dx(da3, W(w_proj, mode).view(Cout, mid))
        del da3
        if ctx.fused:
            # SE backward + BN2/GELU backward in two passes over (dh3, a2); no dh2 in HBM
            da2, dz2, dz1 = K.se_bn_bwd(dh3, a2, Fr, Ho * Wo, mid, w_fc0.detach(), w_fc2.detach(), gate, h1se,
                                        act2, G(g2), G(b2))
        else:
            dh2, dz2, dz1 = K.se_bwd(dh3, h2, Fr, Ho * Wo, mid, w_fc0.detach(), w_fc2.detach(), gate, h1se)
            del h2
            da2 = K.bn_bwd(dh2, a2, m2, r2, g2.detach(), b2.detach(), True, G(g2), G(b2))
            del dh2
        del dh3
        R = mid // 4
        K.gemm(dz2, h1se, G(w_fc2), mid, R, Fr, 1, 1, mid, R, R, beta=1.0)
        K.gemm(dz1, pooled, G(w_fc0), R, mid, Fr, 1, 1, R, mid, mid, beta=1.0)
        if a1 is None:
            a1 = expand(x)
        if ctx.fused:
            # depthwise + BN0/GELU backward in two passes over (da2, a1); dh1 never stored
            act0 = (m0, r0, g0.detach(), b0.detach(), True)
            da1 = K.dwconv_bn_bwd(da2, a1, act0, w_dw.detach().view(mid, 9), G(w_dw).view(mid, 9), G(g0), G(b0),
                                  Fr, H, Wd, mid, stride=s)
            dh1 = None
        else:
            h1 = K.bn_apply(a1, m0, r0, g0.detach(), b0.detach(), gelu=True)
            dh1 = K.dwconv_bwd(da2, h1, w_dw.detach().view(mid, 9), G(w_dw).view(mid, 9), Fr, H, Wd, mid, s)
            del h1
        del da2
        if dh1 is not None:
            da1 = K.bn_bwd(dh1, a1, m0, r0, g0.detach(), b0.detach(), True, G(g0), G(b0))
            del dh1
        x2d = x.reshape(-1, Cin)
        if xbn is not None:     # B operand bf16(BN(x)) formed on load (no gate)
            K.linear_dw_se(da1, x2d, xbn, None, 0, G(w_exp).view(mid, Cin))
        else:
            K.linear_dw(da1, x2d, G(w_exp).view(mid, Cin))
        dx = K.linear_dx(da1, W(w_exp, mode).view(mid, Cin), residual=dout2d if st.res else None)
        _done(*ctx.params)
        return (dx.view(Fr, H, Wd, Cin),) + (None,) * 12


# ============================================================================ transformer block
class BlockFn(torch.autograd.Function):
    """Pre-norm transformer block used by both the TinyViT encoder
    (TinyViTBlock, tiny_vit.py:108-130: global attention, Mlp with GELU) and the MAE
    decoder (nn.TransformerEncoderLayer(norm_first=True, activation='gelu'),
    mae_vit_adapter.py:40-48).  x: [N*L, C] residual stream (bf16 in the encoder,
    fp32 in the decoder)."""

    @staticmethod
    def forward(ctx, x, st, ln1w, ln1b, wqkv, bqkv, wproj, bproj, ln2w, ln2b, w1, b1, w2, b2):
        mode = st.mode
        act = mode.act
        N, L, H, D = st.N, st.L, st.heads, st.head_dim
        rb = mode.bf16
        ln1, mu1, rs1 = K.layernorm(x, ln1w.detach(), ln1b.detach(), out_dtype=act, eps=st.eps)
        qkv = K.linear(ln1, W(wqkv, mode), bqkv.detach())
        del ln1
        o, lse = K.attn_fwd(qkv, N, L, H, D, st.attn_drop, st.seed_attn)
        x2 = K.linear(o, W(wproj, mode), bproj.detach(), out_dtype=x.dtype, residual=x, round_branch=rb,
                      drop_p=st.drop1, seed=st.seed1, row_scale=st.dp1, rows_per_group=L)
        ln2, mu2, rs2 = K.layernorm(x2, ln2w.detach(), ln2b.detach(), out_dtype=act, eps=st.eps)
        h, hpre = K.linear(ln2, W(w1, mode), b1.detach(), gelu=True, drop_p=st.drop_ff, seed=st.seed_ff)
        del ln2
        out = K.linear(h, W(w2, mode), b2.detach(), out_dtype=x.dtype, residual=x2, round_branch=rb,
                       drop_p=st.drop2, seed=st.seed2, row_scale=st.dp2, rows_per_group=L)
        del h
        ctx.st = st
        ctx.params = (ln1w, ln1b, wqkv, bqkv, wproj, bproj, ln2w, ln2b, w1, b1, w2, b2)
        ctx.save_for_backward(x, mu1, rs1, qkv, o, lse, x2, mu2, rs2, hpre)
        return out

    @staticmethod
    def backward(ctx, dout):
        x, mu1, rs1, qkv, o, lse, x2, mu2, rs2, hpre = ctx.saved_tensors
        ln1w, ln1b, wqkv, bqkv, wproj, bproj, ln2w, ln2b, w1, b1, w2, b2 = ctx.params
        st = ctx.st
        mode = st.mode
        act = mode.act
        rb = mode.bf16
        N, L, H, D = st.N, st.L, st.heads, st.head_dim
        _touch(*ctx.params)
        dout = dout.contiguous()
        if dout.dtype != x.dtype:
            dout = dout.to(x.dtype)
        regs2 = st.drop2 > 0 or st.dp2 is not None
        if dout.dtype == torch.float32 and act == torch.bfloat16 and regs2:
            db = K.cast_dropout_bwd(dout, st.drop2, st.seed2, st.dp2, L)   # cast + dropout in one pass
        else:
            db = dout if dout.dtype == act else K.cast(dout, act)       # grad of the bf16 branch
            if regs2:
                db = K.dropout_bwd(db, st.drop2, st.seed2, st.dp2, L)
        # dL/dhpre straight from the fc2 data-gradient GEMM's epilogue (keep mask and
        # GELU' applied there: no dh round trip, no gelu_bwd pass)
        if rb and db.shape[1] <= 256:
            # one-m-tile fc2 weight gradient: dropout(GELU(hpre)) formed in its operand loads
            K.linear_dw_bias(db, hpre, G(w2), G(b2), gelu=(st.drop_ff, st.seed_ff))
            dhpre = K.linear_dx(db, W(w2, mode), gelu_pre=hpre, drop_p=st.drop_ff, seed=st.seed_ff)
        elif rb:   # h = dropout(GELU(hpre)) as a side output of the dX epilogue (hpre read once)
            dhpre, h = K.linear_dx_gelu(db, W(w2, mode), hpre, st.drop_ff, st.seed_ff)
            K.linear_dw_bias(db, h, G(w2), G(b2))
            del h
        else:
            h = K.gelu(hpre, st.drop_ff, st.seed_ff)
            K.linear_dw_bias(db, h, G(w2), G(b2))
            del h
            dhpre = K.linear_dx(db, W(w2, mode), gelu_pre=hpre, drop_p=st.drop_ff, seed=st.seed_ff)
        del db
        ln2 = K.layernorm(x2, ln2w.detach(), ln2b.detach(), out_dtype=act, eps=st.eps)[0]
        K.linear_dw_bias(dhpre, ln2, G(w1), G(b1))
        del ln2
        dln2 = K.linear_dx(dhpre, W(w1, mode))
        del dhpre
        regs1 = st.drop1 > 0 or st.dp1 is not None
        C = x2.shape[1]
        if act == torch.bfloat16 and C in (192, 384) and x2.dtype != act:
            # fp32 stream (decoder): the branch's bf16 copy of dx (cast + dropout backward)
            # from the LayerNorm backward's own pass.  (On the bf16 encoder stream, where only
            # the DropPath scale remains, the separate pass measured cheaper.)
            dx2, dxb = K.layernorm_bwd_branch(dln2, x2, mu2, rs2, ln2w.detach(), G(ln2w), G(ln2b), dres=dout,
                                              drop_p=st.drop1, seed=st.seed1, row_scale=st.dp1, rows_per_group=L)
            del dln2
        else:
            dx2 = K.layernorm_bwd(dln2, x2, mu2, rs2, ln2w.detach(), G(ln2w), G(ln2b), dres=dout)
            del dln2
            dxb = dx2 if dx2.dtype == act else K.cast(dx2, act)
            if regs1:
                dxb = K.dropout_bwd(dxb, st.drop1, st.seed1, st.dp1, L)
        K.linear_dw_bias(dxb, o, G(wproj), G(bproj))
        do = K.linear_dx(dxb, W(wproj, mode))
        del dxb
        dqkv = K.attn_bwd(qkv, o, do, lse, N, L, H, D, st.attn_drop, st.seed_attn)
        del do
        ln1 = K.layernorm(x, ln1w.detach(), ln1b.detach(), out_dtype=act, eps=st.eps)[0]
        K.linear_dw_bias(dqkv, ln1, G(wqkv), G(bqkv))
        del ln1
        dln1 = K.linear_dx(dqkv, W(wqkv, mode))
        del dqkv
        dx = K.layernorm_bwd(dln1, x, mu1, rs1, ln1w.detach(), G(ln1w), G(ln1b), dres=dx2)
        _done(*ctx.params)
        return (dx,) + (None,) * 13


# ============================================================================ enc_to_dec + blend
class EncToDecFn(torch.autograd.Function):
    """enc_to_dec Linear + temporal/spatial pos-embed + mask-token blend
    (mae_vit_adapter.py:90-107).  lat [F*L, 384] -> x [B*T*L, D] fp32."""

    @staticmethod
    def forward(ctx, lat, mask_u8, st, w, b, tpos, spos, tok):
        mode = st.mode
        B, T, L, D = st.B, st.T, st.L, st.D
        y = K.linear(lat, W(w, mode), b.detach())
        x = K.pos_blend(y, tpos.detach().reshape(-1, D), spos.detach().reshape(L, D), tok.detach().reshape(D),
                        mask_u8, B, T, L, D, torch.float32)
        ctx.st = st
        ctx.params = (w, b, tpos, spos, tok)
        ctx.save_for_backward(lat, mask_u8)
        return x

    @staticmethod
    def backward(ctx, dx):
        lat, mask_u8 = ctx.saved_tensors
        w, b, tpos, spos, tok = ctx.params
        st = ctx.st
        mode = st.mode
        B, T, L, D = st.B, st.T, st.L, st.D
        _touch(*ctx.params)
        dx = dx.float().contiguous()
        dy = K.pos_blend_bwd(dx, mask_u8, mode.act, G(tpos).reshape(-1, D), G(spos).reshape(L, D),
                             G(tok).reshape(D), B, T, L, D)
        K.linear_dw_bias(dy, lat, G(w), G(b))
        dlat = K.linear_dx(dy, W(w, mode))
        _done(*ctx.params)
        return dlat, None, None, None, None, None, None, None


# ============================================================================ head
class HeadFn(torch.autograd.Function):
    """decoder_norm + decoder_pred (mae_vit_adapter.py:111-115): x [M, D] -> pred [M, 192]."""

    @staticmethod
    def forward(ctx, x, st, lnw, lnb, w, b):
        mode = st.mode
        ln, mu, rs = K.layernorm(x, lnw.detach(), lnb.detach(), out_dtype=mode.act)
        pred = K.linear(ln, W(w, mode), b.detach())
        ctx.st = st
        ctx.params = (lnw, lnb, w, b)
        ctx.save_for_backward(x, mu, rs)
        return pred

    @staticmethod
    def backward(ctx, dpred):
        x, mu, rs = ctx.saved_tensors
        lnw, lnb, w, b = ctx.params
        mode = ctx.st.mode
        _touch(*ctx.params)
        dpred = dpred.to(mode.act).contiguous()
        ln = K.layernorm(x, lnw.detach(), lnb.detach(), out_dtype=mode.act)[0]
        K.linear_dw_bias(dpred, ln, G(w), G(b))
        del ln
        dln = K.linear_dx(dpred, W(w, mode))
        dx = K.layernorm_bwd(dln, x, mu, rs, lnw.detach(), G(lnw), G(lnb))
        _done(*ctx.params)
        return dx, None, None, None, None, None


# ============================================================================ loss
class MAELossFn(torch.autograd.Function):
    """patchify + norm_pix (unbiased var) + masked MSE (train_ssl_mae.py:26-31,74-84),
    fused; the target never exists in HBM."""

    @staticmethod
    def forward(ctx, pred, clip, mask_u8, norm_pix):
        clip = clip if clip.dtype == torch.float32 else clip.float()
        loss, denom = K.mae_loss_fwd(pred.contiguous(), clip, mask_u8, norm_pix)
        ctx.norm_pix = norm_pix
        ctx.save_for_backward(pred, clip, mask_u8, denom)
        return loss

    @staticmethod
    def backward(ctx, g):
        pred, clip, mask_u8, denom = ctx.saved_tensors
        dpred = K.mae_loss_bwd(pred.contiguous(), clip, mask_u8, ctx.norm_pix, g, denom)
        return dpred, None, None, None


def mae_loss(pred, clip, mask, norm_pix=True):
    """Masked normalised-pixel MSE of the reference (train_ssl_mae.py:72-84)."""
    m = mask if mask.dtype == torch.uint8 else mask.to(torch.uint8)
    if m.device != pred.device:
        m = m.to(pred.device)
    if clip.device != pred.device:
        clip = clip.to(pred.device)
    return MAELossFn.apply(pred, clip, m.contiguous(), bool(norm_pix))


def masked_pred_std(pred, mask_idx):
    """pred[mask.bool()].std() (train_ssl_mae.py:105) from the compacted index list."""
    rows = K.gather_rows(pred.reshape(-1, pred.shape[-1]), mask_idx)
    return K.std(rows)
