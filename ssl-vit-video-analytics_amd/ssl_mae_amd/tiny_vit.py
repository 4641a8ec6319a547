"""TinyViT encoder (reference: src/models/tiny_vit.py), MI355X-native.

Same constructor signatures, module tree and state_dict keys as the reference
(`tiny_vit_21m_variant`, `TinyViT(img_size, in_chans, embed_dims, depths, num_heads,
window_sizes, drop_path_rate, use_checkpoint)`, `forward_stage3`), so reference
checkpoints load unchanged.  The torch sub-modules (nn.Conv2d / nn.BatchNorm2d /
nn.Linear / nn.LayerNorm) are kept only as parameter/buffer containers with the
reference's initialisation; compute runs through the fused HIP Functions of
functions.py on channels-last activations ([frames][H][W][C]), so the reference's
NCHW<->NLC transposes (tiny_vit.py:122,129) do not exist.
"""
import torch
import torch.nn as nn
import torch.utils.checkpoint as checkpoint

from . import ops as K    # every kernel launch through the torch.ops.ssl_mae dispatcher
from .functions import BlockFn, MBConvFn, Mode, StemFn


class DropPath(nn.Module):
    """Stochastic depth (timm.layers.DropPath semantics: per-sample keep with
    probability 1-p, E[mask * scale] = 1); applied inside the fused kernels as a
    per-row-group scale of the residual branch.  The keep test is the counter hash's
    8-bit threshold round(256 p), so kept samples are scaled by 256 / (256 - round(256 p)),
    the inverse of the quantised keep rate (csrc/common.h drop_scale)."""

    def __init__(self, drop_prob=0.0):
        super().__init__()
        self.drop_prob = drop_prob


def droppath_scale(module, n_samples, mode, site, device):
    """Per-sample branch scale for this forward, or None when inactive."""
    dp = getattr(module, "drop_path", None)
    p = getattr(dp, "drop_prob", 0.0) if dp is not None else 0.0
    if not module.training or p <= 0.0:
        return None
    return K.droppath_scale(n_samples, p, mode.seed(getattr(module, "_sm_index", 0), site), device)


class _St:
    """Static per-call configuration handed to a Function (non-tensor)."""

    def __init__(self, **kw):
        self.__dict__.update(kw)


class Conv2d_BN(nn.Sequential):
    """tiny_vit.py:12-18."""

    def __init__(self, a, b, ks=1, stride=1, pad=0, dilation=1, groups=1, bn_weight_init=1):
        super().__init__()
        self.add_module("c", nn.Conv2d(a, b, ks, stride, pad, dilation, groups, bias=False))
        self.add_module("bn", nn.BatchNorm2d(b))
        nn.init.constant_(self.bn.weight, bn_weight_init)
        nn.init.constant_(self.bn.bias, 0)


class SELayer(nn.Module):
    """tiny_vit.py:20-34 (parameters only; fused into MBConvFn)."""

    def __init__(self, channel, reduction=4):
        super().__init__()
        self.avg_pool = nn.AdaptiveAvgPool2d(1)
        self.fc = nn.Sequential(nn.Linear(channel, channel // reduction, bias=False), nn.ReLU(inplace=True),
                                nn.Linear(channel // reduction, channel, bias=False), nn.Sigmoid())


class MBConv(nn.Module):
    """tiny_vit.py:36-56."""

    def __init__(self, in_chans, out_chans, expand_ratio=4, stride=1, drop_path=0.0):
        super().__init__()
        mid = int(in_chans * expand_ratio)
        if expand_ratio != 4:
            raise NotImplementedError("only expand_ratio=4 (the reference's only use) is fused")
        self.in_chans, self.out_chans, self.mid, self.stride = in_chans, out_chans, mid, stride
        self.use_res_connect = stride == 1 and in_chans == out_chans
        self.conv = nn.Sequential(
            Conv2d_BN(in_chans, mid, ks=1), nn.GELU(),
            Conv2d_BN(mid, mid, ks=3, stride=stride, pad=1, groups=mid), nn.GELU(),
            SELayer(mid),
            Conv2d_BN(mid, out_chans, ks=1, bn_weight_init=0))
        self.drop_path = DropPath(drop_path) if drop_path > 0.0 else nn.Identity()

    def run(self, x, mode, resident=False, x_bn=None):
        c = self.conv
        dps = droppath_scale(self, x.shape[0], mode, 0, x.device) if self.use_res_connect else None
        st = _St(mode=mode, mid=self.mid, cout=self.out_chans, stride=self.stride, res=self.use_res_connect,
                 bn0=c[0].bn, bn2=c[2].bn, bn5=c[5].bn, dp_scale=dps, bn_updates=2 if resident else 1,
                 recompute_a1=bool(resident), recompute_a2=resident == "lite", x_bn=x_bn)
        return MBConvFn.apply(x, st, c[0].c.weight, c[0].bn.weight, c[0].bn.bias, c[2].c.weight, c[2].bn.weight,
                              c[2].bn.bias, c[4].fc[0].weight, c[4].fc[2].weight, c[5].c.weight, c[5].bn.weight,
                              c[5].bn.bias)


class PatchEmbed(nn.Module):
    """tiny_vit.py:62-72: conv3x3 s2 -> BN -> GELU -> conv3x3 s1 -> BN."""

    def __init__(self, in_chans, embed_dim):
        super().__init__()
        self.patch_embed = nn.Sequential(
            Conv2d_BN(in_chans, embed_dim // 2, ks=3, stride=2, pad=1), nn.GELU(),
            Conv2d_BN(embed_dim // 2, embed_dim, ks=3, stride=1, pad=1))

    # BN2's apply folded into stages[0][0] when the stem runs its direct conv2 (bf16
    # training): False keeps the stored y = BN2(a2) (bit-identical either way)
    fold_bn2 = True

    def run(self, clip, mode, fold_ok=True):
        """-> (t, x_bn): t the stem output, or with x_bn = (mean, rstd, weight, bias) of BN2
        the conv2 output a2 that stages[0][0] reads as bf16(BN2(a2)) (StemFn).  fold_ok: the
        consumer can take the folded form (TinyViT._stem_fold_ok)."""
        pe = self.patch_embed
        if pe[0].c.weight.shape[:2] != (48, 3) or pe[2].c.weight.shape[:2] != (96, 48):
            raise NotImplementedError("fused stem is specialised for 3->48->96 (embed_dims[0]=96)")
        bn1, bn2 = pe[0].bn, pe[2].bn
        wo = (clip.shape[-1] - 1) // 2 + 1
        fold = bool(self.fold_bn2) and fold_ok and mode.bf16 and bn1.training and bn2.training and wo <= 128
        st = _St(mode=mode, bn1=bn1, bn2=bn2, fold_bn2=fold)
        t, m2, r2 = StemFn.apply(clip, st, pe[0].c.weight, bn1.weight, bn1.bias, pe[2].c.weight, bn2.weight,
                                 bn2.bias)
        return t, ((m2, r2, bn2.weight.detach(), bn2.bias.detach()) if fold else None)


class Mlp(nn.Module):
    """tiny_vit.py:74-84."""

    def __init__(self, in_features, hidden_features=None, out_features=None, act_layer=nn.GELU, drop=0.0):
        super().__init__()
        out_features = out_features or in_features
        hidden_features = hidden_features or in_features
        self.fc1 = nn.Linear(in_features, hidden_features)
        self.act = act_layer()
        self.fc2 = nn.Linear(hidden_features, out_features)
        self.drop = nn.Dropout(drop)


class Attention(nn.Module):
    """tiny_vit.py:86-106 (global softmax attention over all tokens)."""

    def __init__(self, dim, key_dim, num_heads=8, window_size=7):
        super().__init__()
        self.num_heads = num_heads
        self.scale = key_dim ** -0.5
        self.key_dim = key_dim
        self.qkv = nn.Linear(dim, key_dim * num_heads * 3)
        self.proj = nn.Linear(key_dim * num_heads, dim)


class TinyViTBlock(nn.Module):
    """tiny_vit.py:108-130 (window_size accepted and ignored, as in the reference)."""

    def __init__(self, dim, num_heads, window_size=7, mlp_ratio=4.0, drop_path=0.0):
        super().__init__()
        self.dim, self.num_heads = dim, num_heads
        self.norm1 = nn.LayerNorm(dim)
        self.attn = Attention(dim, key_dim=dim // num_heads, num_heads=num_heads, window_size=window_size)
        self.drop_path = DropPath(drop_path) if drop_path > 0.0 else nn.Identity()
        self.norm2 = nn.LayerNorm(dim)
        self.mlp = Mlp(in_features=dim, hidden_features=int(dim * mlp_ratio))

    def run(self, x, mode, resident=False):   # no BatchNorm, nothing to trade: resident unused
        Fr, H, Wd, C = x.shape
        st = _St(mode=mode, N=Fr, L=H * Wd, heads=self.num_heads, head_dim=C // self.num_heads,
                 eps=self.norm1.eps, attn_drop=0.0, seed_attn=0, drop1=0.0, seed1=0, drop_ff=0.0, seed_ff=0,
                 drop2=0.0, seed2=0, dp1=droppath_scale(self, Fr, mode, 1, x.device),
                 dp2=droppath_scale(self, Fr, mode, 2, x.device))
        a, m = self.attn, self.mlp
        y = BlockFn.apply(x.reshape(Fr * H * Wd, C), st, self.norm1.weight, self.norm1.bias, a.qkv.weight,
                          a.qkv.bias, a.proj.weight, a.proj.bias, self.norm2.weight, self.norm2.bias,
                          m.fc1.weight, m.fc1.bias, m.fc2.weight, m.fc2.bias)
        return y.view(Fr, H, Wd, C)


class _Stage(nn.Sequential):
    def run(self, x, mode, resident=False, x_bn=None):
        """x_bn: x is stored before its BatchNorm (stage 0 under the stem's folded BN2):
        only the first block reads it."""
        for i, blk in enumerate(self):
            if i == 0 and x_bn is not None:
                x = blk.run(x, mode, resident, x_bn=x_bn)
            else:
                x = blk.run(x, mode, resident)
        return x


class TinyViT(nn.Module):
    """tiny_vit.py:136-186."""

    def __init__(self, img_size=112, in_chans=3, embed_dims=[96, 192, 384, 576], depths=[2, 2, 6, 2],
                 num_heads=[3, 6, 12, 24], window_sizes=[7, 7, 14, 7], drop_path_rate=0.1, use_checkpoint=True):
        super().__init__()
        self.use_checkpoint = use_checkpoint
        # Stages whose activations stay resident in HBM instead of being dropped and
        # recomputed under use_checkpoint (see _run_stages): a tuple, or "auto"
        # (auto_resident_stages: as many as the device memory holds).
        self.resident_stages = "auto"
        # Stages kept "lite-resident": only block inputs / outputs and statistics are
        # kept; the two largest tensors of each MBConv are recomputed in its backward
        # instead of re-running the whole stage forward (stage 0: the 112x112 MBConvs).
        self.lite_stages = "auto"
        self.embed_dims = list(embed_dims)
        self.depths = list(depths)
        self._sm_dec_depth = 4          # set by TinyVideoMAE (memory policy key)
        self.patch_embed = PatchEmbed(in_chans, embed_dims[0])
        self.stages = nn.ModuleList()
        dpr = [x.item() for x in torch.linspace(0, drop_path_rate, sum(depths))]
        cur = 0
        for i in range(4):
            blocks = []
            if i > 0:
                blocks.append(MBConv(embed_dims[i - 1], embed_dims[i], stride=2))
            for j in range(depths[i]):
                if i == 0:
                    blocks.append(MBConv(embed_dims[i], embed_dims[i], drop_path=dpr[cur]))
                else:
                    blocks.append(TinyViTBlock(dim=embed_dims[i], num_heads=num_heads[i],
                                               window_size=window_sizes[i], drop_path=dpr[cur]))
                cur += 1
            self.stages.append(_Stage(*blocks))
        index_modules(self)

    # ------------------------------------------------------------------ internals
    def _mode(self):
        from .mae_vit_adapter import next_seed_base
        return Mode(torch.is_autocast_enabled("cuda"), next_seed_base(self))

    def _run_stages(self, x, n_stages, mode, x_bn=None):
        """tiny_vit.py:170-175: each stage under checkpoint(use_reentrant=False) when
        training with use_checkpoint.  A stage listed in resident_stages keeps its
        activations in HBM instead (288 GB holds them at the bench batch): no
        recompute, and its BatchNorms take the batch statistics twice, which is what
        the reference's checkpoint forward + recompute does to the running stats
        (num_batches_tracked += 2).  Every output, gradient and buffer is identical;
        only the memory/time trade changes.  (An MBConv in a resident stage still
        drops its 4x-wide expand output and recomputes that one GEMM.)"""
        resident = self.resident_stages
        # Without autograd (frozen encoder, no_grad evaluation) the reference's
        # non-reentrant checkpoint runs each stage's forward once and never recomputes
        # it, so BatchNorm takes the batch once: plain forward here too.
        grad = torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in self.parameters()))
        lite = self.lite_stages
        key = (tuple(self.depths), self._sm_dec_depth)
        if resident == "auto":
            resident = auto_resident_stages(x.shape[0], x.shape[1] * 2, mode.bf16, x.device, key=key) \
                if self.use_checkpoint and self.training and grad else ()
        explicit = self.resident_stages != "auto" or lite != "auto"
        if lite == "auto":
            lite = auto_lite_stages(x.shape[0], x.shape[1] * 2, mode.bf16, x.device, resident, key=key) \
                if self.use_checkpoint and self.training and grad else ()
        if explicit and self.use_checkpoint and self.training and grad:
            check_memory_policy(x.shape[0], x.shape[1] * 2, mode.bf16, x.device, resident, lite, key=key)
        for i in range(n_stages):
            stage = self.stages[i]
            xb = x_bn if i == 0 else None
            if self.use_checkpoint and self.training and grad:
                if i in resident:
                    x = stage.run(x, mode, True, xb)
                elif i in lite:
                    x = stage.run(x, mode, "lite", xb)
                else:
                    x = checkpoint.checkpoint(stage.run, x, mode, False, xb, use_reentrant=False)
            else:
                x = stage.run(x, mode, False, xb)
        return x

    def _stem_fold_ok(self):
        """The stem's BN2 fold needs a consumer that forms bf16(BN2(a2)) in its loads: a fused
        MBConv first block (the BatchNorm-input expand GEMM: mid % 32 == 0, <= 256 input
        channels); anything else takes the stem's stored output."""
        blk = self.stages[0][0] if len(self.stages[0]) else None
        return isinstance(blk, MBConv) and blk.mid % 32 == 0 and blk.in_chans <= 256

    def tokens_stage3(self, clip, mode):
        """clip [B,3,T,H,W] or frames [N,3,H,W] -> channels-last [N*T, H/8, W/8, 384]."""
        x, x_bn = self.patch_embed.run(clip, mode, self._stem_fold_ok())
        return self._run_stages(x, 3, mode, x_bn)

    def _prepare(self, mode):
        from .mae_vit_adapter import ensure_flat
        ensure_flat(self, mode)

    # ------------------------------------------------------------------ reference API
    def forward_stage3(self, x):
        """MAE entry point (tiny_vit.py:166-176): [N,3,H,W] -> [N,384,H/8,W/8] (NCHW view)."""
        mode = self._mode()
        self._prepare(mode)
        t = self.tokens_stage3(x, mode)
        return t.permute(0, 3, 1, 2)

    def tokens_all(self, x, mode):
        """All four stages, channels-last: frames [N,3,H,W] (any strides) or a clip
        [B,3,T,H,W] (frames b*T + t) -> [N, H/16, W/16, C4]."""
        t, x_bn = self.patch_embed.run(x, mode, self._stem_fold_ok())
        return self._run_stages(t, 4, mode, x_bn)

    def forward(self, x):
        """All four stages (tiny_vit.py:178-186) -> [N, C4, H/16, W/16] (NCHW view)."""
        mode = self._mode()
        self._prepare(mode)
        return self.tokens_all(x, mode).permute(0, 3, 1, 2)


# Peak HBM of one MAE training step per frame (GiB, bf16, 224x224 frames, measured
# with bench.py at B=256 clips x T=8 on MI355X) for each resident-stage policy, per
# (encoder depths, decoder depth); activations scale with the pixel count, fp32
# doubles them.  An unlisted model takes the reference's policy (all checkpointed).
_PEAK_GIB_PER_FRAME = {
    # (0, 1, 2): stage 0 resident too, 2 x 131.9 GiB at B = 128 less the B-independent 0.7 GiB
    ((2, 2, 6, 2), 4): {(0, 1, 2): 263.1 / 2048, (1, 2): 216.0 / 2048, (2,): 171.9 / 2048, (): 143.6 / 2048},
    # C3 ViT-Small (depths 2,2,12,2 + 8-layer decoder): (2,) and (1, 2) exceed 288 GB at B=256;
    # (0,) (stage 0 resident, arena only) 231.2 GiB, +3.2 % (profiles/r05ap_small_stage0_resident.txt)
    ((2, 2, 12, 2), 8): {(0,): 231.2 / 2048, (): 184.0 / 2048},
}


# Policies measured to run out of memory at B = 256 (GiB per frame: the memory in use when the
# failing request arrived plus that request, a LOWER bound on the policy's peak).  C3 ViT-Small
# with stage 2 resident: 295.1 GB in use + a 4.9 GB request (profiles/r05ap_small_stage0_resident.txt).
_PEAK_LOWER_BOUND_GIB_PER_FRAME = {((2, 2, 12, 2), 8): {(2,): (295123654656 + 4932501504) / 2 ** 30 / 2048}}


def predicted_peak_gib(frames, image_size, bf16, resident, lite=(), key=((2, 2, 6, 2), 4)):
    """(GiB, basis) of one training step's peak under a resident / lite policy, from the
    measured tables: basis "measured", "lower bound" (the policy, or a subset of it, was
    measured out of memory) or "estimate" (the all-checkpointed peak plus per-block stage
    costs taken from the TinyViT-21M measurements); (None, None) for an unmeasured model."""
    resident, lite = tuple(sorted(resident)), tuple(sorted(lite))
    scale = frames * (image_size / 224.0) ** 2 * (1 if bf16 else 2)
    table = _PEAK_GIB_PER_FRAME.get(key)
    if table is None:
        return None, None
    extra = 0.0
    if lite:
        e = _LITE0_EXTRA_GIB_PER_FRAME.get((key, resident))
        extra = e if e is not None else 0.0
    if resident in table:
        return (table[resident] + extra) * scale, "measured"
    lb = _PEAK_LOWER_BOUND_GIB_PER_FRAME.get(key, {})
    bounds = [v for pol, v in lb.items() if set(pol) <= set(resident)]
    if bounds:
        return max(bounds) * scale, "lower bound"
    if () not in table:
        return None, None
    t = _PEAK_GIB_PER_FRAME[((2, 2, 6, 2), 4)]
    per_block = {2: (t[(2,)] - t[()]) / 6, 1: (t[(1, 2)] - t[(2,)]) / 2, 0: (t[(0, 1, 2)] - t[(1, 2)]) / 2}
    depths = key[0]
    est = table[()] + sum(per_block[s] * depths[s] for s in resident if s in per_block)
    return (est + extra) * scale, "estimate"


def check_memory_policy(frames, image_size, bf16, device, resident, lite=(), key=((2, 2, 6, 2), 4),
                        arena_budget=0.96):
    """Raise RuntimeError before the step when an explicitly requested resident / lite policy
    cannot fit: its predicted peak (predicted_peak_gib) against `arena_budget` of the
    device-memory arena's capacity (the rest is fragmentation headroom: the measured C3
    stage-2 failure met a 4.6 GiB request with 6.5 GiB free but split), or, under the caching
    allocator, the device's total memory.  The arena would otherwise meet the failing request
    deep inside the step, where PyTorch's pluggable-allocator hook cannot turn it into an
    exception (csrc/arena.cpp stops the process with the sizes)."""
    pred, basis = predicted_peak_gib(frames, image_size, bf16, resident, lite, key)
    if pred is None:
        return
    from . import arena
    cap = arena.capacity_gib(device) if arena.active() else 0.0
    if cap:
        limit, what = arena_budget * cap, f"{arena_budget:.0%} of the device-memory arena's {cap:.1f} GiB"
    else:
        limit = torch.cuda.get_device_properties(device).total_memory / 2 ** 30
        what = f"the device's {limit:.1f} GiB"
    if pred > limit:
        raise RuntimeError(
            f"memory policy resident_stages={tuple(resident)} lite_stages={tuple(lite)} needs {pred:.1f} GiB "
            f"({basis}) for {frames} frames of {image_size}x{image_size}, more than {what} ({limit:.1f} GiB); "
            f"use fewer resident stages (or resident_stages='auto')")


def auto_resident_stages(frames, image_size, bf16, device, budget=0.85, key=((2, 2, 6, 2), 4),
                         arena_budget=0.96):
    """The largest resident set whose predicted step peak fits `budget` of the
    device memory.  Stage 0 (the 112x112 MBConvs) is resident only under the
    device-memory arena (ssl_mae_amd/arena.py) and when the prediction fits
    `arena_budget` of its capacity: the caching allocator's exact-size segments
    leave ~50 GB of slack at B = 256, which the 263 GiB of that policy do not
    survive (profiles/r05ik_allocator_policy.txt)."""
    table = _PEAK_GIB_PER_FRAME.get(key)
    if table is None:
        return ()
    total = torch.cuda.get_device_properties(device).total_memory / 2 ** 30
    scale = frames * (image_size / 224.0) ** 2 * (1 if bf16 else 2)
    for policy in ((0, 1, 2), (1, 2), (2,), (0,)):
        if policy not in table:
            continue
        if 0 in policy:
            from . import arena
            cap = arena.capacity_gib(device) if arena.active() else 0.0
            if cap and table[policy] * scale <= arena_budget * cap:
                return policy
        elif table[policy] * scale <= budget * total:
            return policy
    return ()


# Extra peak per frame of keeping stage 0 lite-resident, on top of the resident policy
# (GiB, measured like _PEAK_GIB_PER_FRAME); absent: not measured -> not used.
_LITE0_EXTRA_GIB_PER_FRAME = {(((2, 2, 6, 2), 4), (1, 2)): 13.8 / 2048}   # 216.0 -> 229.8 GiB at B=256


def auto_lite_stages(frames, image_size, bf16, device, resident, budget=0.92, key=((2, 2, 6, 2), 4)):
    table = _PEAK_GIB_PER_FRAME.get(key)
    extra = _LITE0_EXTRA_GIB_PER_FRAME.get((key, tuple(resident)))
    if table is None or extra is None or tuple(resident) not in table:
        return ()
    total = torch.cuda.get_device_properties(device).total_memory / 2 ** 30
    scale = frames * (image_size / 224.0) ** 2 * (1 if bf16 else 2)
    return (0,) if (table[tuple(resident)] + extra) * scale <= budget * total else ()


def index_modules(root):
    """Stable per-module indices for the dropout/DropPath seed derivation."""
    for i, m in enumerate(root.modules()):
        m._sm_index = i


def tiny_vit_21m_variant(img_size=112, use_checkpoint=True, **kwargs):
    """tiny_vit.py:188-191."""
    return TinyViT(img_size=img_size, embed_dims=[96, 192, 384, 576], depths=[2, 2, 6, 2],
                   num_heads=[3, 6, 12, 18], use_checkpoint=use_checkpoint, **kwargs)


def tiny_vit_small_variant(img_size=112, use_checkpoint=True, **kwargs):
    """BASELINE config 3 "ViT-Small" MAE encoder.  The reference has no Small model
    (SURVEY.md H8); this is the build-defined variant of the reference's parametric
    TinyViT (tiny_vit.py:137-140) that keeps the stage-3 width TinyVideoMAE hard-codes
    (encoder_dim = 384, mae_vit_adapter.py:18): depths (2, 2, 12, 2) instead of
    (2, 2, 6, 2); pair it with decoder_depth 8 in the MAE config."""
    return TinyViT(img_size=img_size, embed_dims=[96, 192, 384, 576], depths=[2, 2, 12, 2],
                   num_heads=[3, 6, 12, 18], use_checkpoint=use_checkpoint, **kwargs)


ENCODERS = {"tiny_vit_21m_variant": tiny_vit_21m_variant, "tiny_vit_small_variant": tiny_vit_small_variant}
