"""CPU ORACLE — TEST INFRASTRUCTURE ONLY.

A from-scratch fp32 CPU restatement (torch CPU ops, functional form) of the
reference's MAE pretraining step.  Only `tests/`, `__graft_entry__.smoke()` and the
`cpu_baseline` leg of `bench.py` may import this module, and only as the checker /
CPU baseline — the product path (ssl_mae_amd) never imports it.

Pinned against golden fixtures produced by RUNNING the reference in the build
container (`tests/golden/make_golden.py`; checked by `tests/test_oracle_golden.py`).

What it follows (reference file:line, relative to the reference repo root):
  get_tube_mask          src/datasets/mae_loader.py:80-90
  patchify               src/train_ssl_mae.py:26-31
  norm_pix target        src/train_ssl_mae.py:74-77   (unbiased var, eps 1e-6)
  masked MSE             src/train_ssl_mae.py:81-84
  Conv2d_BN              src/models/tiny_vit.py:12-18 (train-mode BN, eps 1e-5, momentum 0.1)
  SELayer                src/models/tiny_vit.py:20-34
  MBConv                 src/models/tiny_vit.py:36-56
  PatchEmbed             src/models/tiny_vit.py:62-72
  Mlp / Attention        src/models/tiny_vit.py:74-106
  TinyViTBlock           src/models/tiny_vit.py:108-130
  forward_stage3         src/models/tiny_vit.py:166-176 (stages 0-2 checkpointed: BN
                         running stats of stages 0-2 updated twice per step)
  TinyVideoMAE.forward   src/models/mae_vit_adapter.py:75-117
  decoder layer          torch nn.TransformerEncoderLayer(norm_first, gelu, FF 4d)
                         built at src/models/mae_vit_adapter.py:40-48
  AdamW step             src/train_ssl_mae.py:163 (lr from config, wd 0.05, betas
                         (0.9, 0.999), eps 1e-8; params whose grad is None skipped)
Dropout / DropPath are 0 in parity mode.  cfg["train_dropout"] = True
(bench.py's cpu_baseline only, never a parity check) runs them as the reference ships them,
on torch's CPU RNG: the decoder layers' nn.Dropout(0.1) on the attention probabilities, the
attention output, the FF activation and the FF output (torch TransformerEncoderLayer
defaults), and the encoder blocks' DropPath with rates linspace(0, 0.1, 12)
(tiny_vit.py:146-158, timm's per-sample stochastic depth) -- the reference's CPU step
spends ~41 % of its time in those bernoulli draws.
"""
import math

import torch
import torch.nn.functional as F

EMBED = (96, 192, 384, 576)
DEPTHS = (2, 2, 6, 2)          # tiny_vit_21m_variant (tiny_vit.py:188-191)
HEADS = (3, 6, 12, 18)
# BASELINE config 3 "ViT-Small": build-defined, the reference's
# parametric TinyViT (tiny_vit.py:137-140) with depths (2, 2, 12, 2), decoder depth 8
SMALL_DEPTHS = (2, 2, 12, 2)


def depths_of(cfg):
    return tuple(cfg.get("model", {}).get("depths", DEPTHS)) if cfg else DEPTHS


# ---------------------------------------------------------------- masking / target
def get_tube_mask(batch_size, num_frames, num_patches, mask_ratio):
    """mae_loader.py:80-90: per sample torch.rand(L) from the global CPU generator,
    the int(r*L) largest noise positions are masked, repeated over T."""
    n_mask = int(mask_ratio * num_patches)
    rows = torch.zeros(batch_size, num_patches)
    for b in range(batch_size):
        noise = torch.rand(num_patches)
        order = torch.argsort(noise, descending=True)
        rows[b, order[:n_mask]] = 1.0
    return rows[:, None, :].expand(batch_size, num_frames, num_patches).bool().contiguous()


def patchify(imgs, p=8):
    """train_ssl_mae.py:26-31: token (t, h, w), feature (pi, qi, c)."""
    B, C, T, H, W = imgs.shape
    x = imgs.reshape(B, C, T, H // p, p, W // p, p)
    x = x.permute(0, 2, 3, 5, 4, 6, 1)        # b t h w pi qi c
    return x.reshape(B, T * (H // p) * (W // p), p * p * C)


def norm_pix(target):
    mu = target.mean(-1, keepdim=True)
    var = target.var(-1, keepdim=True)          # unbiased (N-1)
    return (target - mu) / torch.sqrt(var + 1e-6)


def masked_mse(pred, target, mask):
    per_tok = ((pred.float() - target) ** 2).mean(-1)
    m = mask.reshape(mask.shape[0], -1).to(per_tok.dtype)
    return (per_tok * m).sum() / (m.sum() + 1e-6)


# ---------------------------------------------------------------- encoder pieces
class _BNTracker:
    """Collects (bn prefix, batch mean, unbiased batch var, count, n_updates)."""

    def __init__(self):
        self.stats = []


def _conv_bn(P, pre, x, stride=1, pad=0, groups=1, trk=None, updates=1):
    y = F.conv2d(x, P[pre + ".c.weight"], None, stride, pad, 1, groups)
    dims = (0, 2, 3)
    mean = y.mean(dims)
    var_b = y.var(dims, unbiased=False)
    n = y.numel() // y.shape[1]
    if trk is not None:
        trk.stats.append((pre + ".bn", mean.detach(), var_b.detach() * n / max(n - 1, 1), updates))
    yhat = (y - mean[None, :, None, None]) / torch.sqrt(var_b[None, :, None, None] + 1e-5)
    return yhat * P[pre + ".bn.weight"][None, :, None, None] + P[pre + ".bn.bias"][None, :, None, None]


def _se(P, pre, x):
    s = x.mean((2, 3))
    s = torch.relu(s @ P[pre + ".fc.0.weight"].t())
    s = torch.sigmoid(s @ P[pre + ".fc.2.weight"].t())
    return x * s[:, :, None, None]


_DROP = {"on": False}


def _drop_path(h, p):
    """timm DropPath (scale_by_keep): per-sample keep with prob 1 - p, kept rows / (1 - p)."""
    if not _DROP["on"] or p <= 0.0:
        return h
    keep = torch.empty((h.shape[0],) + (1,) * (h.dim() - 1)).bernoulli_(1 - p)
    return h * keep / (1 - p)


def _dropout(x, p=0.1):
    return F.dropout(x, p, training=True) if _DROP["on"] else x


def _mbconv(P, pre, x, cin, cout, stride, trk, upd, dp=0.0):
    mid = cin * 4
    h = F.gelu(_conv_bn(P, pre + ".conv.0", x, trk=trk, updates=upd))
    h = F.gelu(_conv_bn(P, pre + ".conv.2", h, stride, 1, mid, trk=trk, updates=upd))
    h = _se(P, pre + ".conv.4", h)
    h = _conv_bn(P, pre + ".conv.5", h, trk=trk, updates=upd)
    if stride == 1 and cin == cout:
        return x + _drop_path(h, dp)
    return h


def _ln(P, pre, x, eps=1e-5):
    return F.layer_norm(x, (x.shape[-1],), P[pre + ".weight"], P[pre + ".bias"], eps)


def _attention_core(q, k, v):
    """softmax(q k^T / sqrt(d)) v on [N, h, L, d]."""
    return F.scaled_dot_product_attention(q, k, v)


def _vit_block(P, pre, x, heads, dp=0.0):
    N, C, H, W = x.shape
    t = x.flatten(2).transpose(1, 2)
    d = C // heads
    h = _ln(P, pre + ".norm1", t)
    qkv = h @ P[pre + ".attn.qkv.weight"].t() + P[pre + ".attn.qkv.bias"]
    qkv = qkv.reshape(N, H * W, 3, heads, d).permute(2, 0, 3, 1, 4)
    a = _attention_core(qkv[0], qkv[1], qkv[2]).transpose(1, 2).reshape(N, H * W, C)
    t = t + _drop_path(a @ P[pre + ".attn.proj.weight"].t() + P[pre + ".attn.proj.bias"], dp)
    h = _ln(P, pre + ".norm2", t)
    h = F.gelu(h @ P[pre + ".mlp.fc1.weight"].t() + P[pre + ".mlp.fc1.bias"])
    t = t + _drop_path(h @ P[pre + ".mlp.fc2.weight"].t() + P[pre + ".mlp.fc2.bias"], dp)
    return t.transpose(1, 2).reshape(N, C, H, W)


def forward_stage3(P, x, trk=None, prefix="encoder.", acts=None, depths=DEPTHS):
    pe = prefix + "patch_embed.patch_embed"
    dpr = torch.linspace(0, 0.1, sum(depths)).tolist()   # TinyViT drop_path_rate 0.1 (tiny_vit.py:146)
    cur = 0
    h = F.gelu(_conv_bn(P, pe + ".0", x, 2, 1, trk=trk, updates=1))
    h = _conv_bn(P, pe + ".2", h, 1, 1, trk=trk, updates=1)
    if acts is not None:
        acts["act_stem"] = h
    for i in range(3):
        sp = f"{prefix}stages.{i}."
        j0 = 0
        if i > 0:
            h = _mbconv(P, sp + "0", h, EMBED[i - 1], EMBED[i], 2, trk, 2)
            j0 = 1
        for j in range(depths[i]):
            if i == 0:
                h = _mbconv(P, sp + str(j0 + j), h, EMBED[0], EMBED[0], 1, trk, 2, dpr[cur])
            else:
                h = _vit_block(P, sp + str(j0 + j), h, HEADS[i], dpr[cur])
            cur += 1
        if acts is not None:
            acts[f"act_stage{i}"] = h
    return h


# ---------------------------------------------------------------- decoder
def _decoder_layer(P, pre, x, heads):
    B, L, D = x.shape
    d = D // heads
    h = _ln(P, pre + ".norm1", x)
    qkv = h @ P[pre + ".self_attn.in_proj_weight"].t() + P[pre + ".self_attn.in_proj_bias"]
    q, k, v = (t.reshape(B, L, heads, d).transpose(1, 2) for t in qkv.split(D, dim=-1))
    if _DROP["on"]:   # nn.MultiheadAttention(dropout=0.1) on the probabilities (explicit, as MHA's math path)
        pr = F.dropout(torch.softmax((q @ k.transpose(-2, -1)) / math.sqrt(d), -1), 0.1, training=True)
        a = (pr @ v).transpose(1, 2).reshape(B, L, D)
    else:
        a = _attention_core(q, k, v).transpose(1, 2).reshape(B, L, D)
    x = x + _dropout(a @ P[pre + ".self_attn.out_proj.weight"].t() + P[pre + ".self_attn.out_proj.bias"])
    h = _ln(P, pre + ".norm2", x)
    h = _dropout(F.gelu(h @ P[pre + ".linear1.weight"].t() + P[pre + ".linear1.bias"]))
    return x + _dropout(h @ P[pre + ".linear2.weight"].t() + P[pre + ".linear2.bias"])


def mae_forward(P, clip, mask, cfg, trk=None, acts=None):
    """TinyVideoMAE.forward (mae_vit_adapter.py:75-117) -> pred [B, T*L, 192]."""
    B, C, T, H, W = clip.shape
    _DROP["on"] = bool(cfg.get("train_dropout", False))
    frames = clip.permute(0, 2, 1, 3, 4).reshape(B * T, C, H, W)
    lat = forward_stage3(P, frames, trk, acts=acts, depths=depths_of(cfg))
    Lp = lat.shape[2] * lat.shape[3]
    tok = lat.flatten(2).transpose(1, 2)
    x = tok @ P["enc_to_dec.weight"].t() + P["enc_to_dec.bias"]
    D = x.shape[-1]
    x = x.reshape(B, T, Lp, D) + (P["temporal_pos_embed"][:, :T] + P["spatial_pos_embed"])
    m = mask.to(x.dtype)[..., None]
    x = x * (1 - m) + P["mask_token"] * m
    x = x.reshape(B, T * Lp, D)
    depth = cfg["model"]["decoder_depth"]
    heads = cfg["model"]["decoder_num_heads"]
    for i in range(depth):
        x = _decoder_layer(P, f"decoder_blocks.layers.{i}", x, heads)
    x = _ln(P, "decoder_norm", x)
    pred = x @ P["decoder_pred.weight"].t() + P["decoder_pred.bias"]
    if acts is not None:
        acts["pred"] = pred
    return pred


# ---------------------------------------------------------------- parameters
def param_shapes(cfg):
    """(name, shape) for every parameter of tiny_vit_21m_variant + TinyVideoMAE."""
    S = cfg["dataset"]["image_size"]
    T = cfg["dataset"]["clip_len"]
    D = cfg["model"]["decoder_embed_dim"]
    depth = cfg["model"]["decoder_depth"]
    out = [("mask_token", (1, 1, D)), ("temporal_pos_embed", (1, T, 1, D)),
           ("spatial_pos_embed", (1, 1, (S // 8) ** 2, D))]

    def conv_bn(pre, cin, cout, k, groups=1):
        out.extend([(pre + ".c.weight", (cout, cin // groups, k, k)),
                    (pre + ".bn.weight", (cout,)), (pre + ".bn.bias", (cout,))])

    def mbconv(pre, cin, cout):
        mid = cin * 4
        conv_bn(pre + ".conv.0", cin, mid, 1)
        conv_bn(pre + ".conv.2", mid, mid, 3, mid)
        out.extend([(pre + ".conv.4.fc.0.weight", (mid // 4, mid)),
                    (pre + ".conv.4.fc.2.weight", (mid, mid // 4))])
        conv_bn(pre + ".conv.5", mid, cout, 1)

    def block(pre, c):
        out.extend([(pre + ".norm1.weight", (c,)), (pre + ".norm1.bias", (c,)),
                    (pre + ".attn.qkv.weight", (3 * c, c)), (pre + ".attn.qkv.bias", (3 * c,)),
                    (pre + ".attn.proj.weight", (c, c)), (pre + ".attn.proj.bias", (c,)),
                    (pre + ".norm2.weight", (c,)), (pre + ".norm2.bias", (c,)),
                    (pre + ".mlp.fc1.weight", (4 * c, c)), (pre + ".mlp.fc1.bias", (4 * c,)),
                    (pre + ".mlp.fc2.weight", (c, 4 * c)), (pre + ".mlp.fc2.bias", (c,))])

    pe = "encoder.patch_embed.patch_embed"
    conv_bn(pe + ".0", 3, EMBED[0] // 2, 3)
    conv_bn(pe + ".2", EMBED[0] // 2, EMBED[0], 3)
    for i in range(4):
        j = 0
        if i > 0:
            mbconv(f"encoder.stages.{i}.0", EMBED[i - 1], EMBED[i])
            j = 1
        for k in range(depths_of(cfg)[i]):
            if i == 0:
                mbconv(f"encoder.stages.{i}.{j + k}", EMBED[0], EMBED[0])
            else:
                block(f"encoder.stages.{i}.{j + k}", EMBED[i])
    out.extend([("enc_to_dec.weight", (D, 384)), ("enc_to_dec.bias", (D,))])
    for i in range(depth):
        pre = f"decoder_blocks.layers.{i}"
        out.extend([(pre + ".self_attn.in_proj_weight", (3 * D, D)),
                    (pre + ".self_attn.in_proj_bias", (3 * D,)),
                    (pre + ".self_attn.out_proj.weight", (D, D)),
                    (pre + ".self_attn.out_proj.bias", (D,)),
                    (pre + ".linear1.weight", (4 * D, D)), (pre + ".linear1.bias", (4 * D,)),
                    (pre + ".linear2.weight", (D, 4 * D)), (pre + ".linear2.bias", (D,)),
                    (pre + ".norm1.weight", (D,)), (pre + ".norm1.bias", (D,)),
                    (pre + ".norm2.weight", (D,)), (pre + ".norm2.bias", (D,))])
    out.extend([("decoder_norm.weight", (D,)), ("decoder_norm.bias", (D,)),
                ("decoder_pred.weight", (192, D)), ("decoder_pred.bias", (192,))])
    return out


def make_params(cfg, rule):
    return {n: torch.from_numpy(rule(n, s)).clone() for n, s in param_shapes(cfg)}


# ---------------------------------------------------------------- training step
class AdamWState:
    """torch.optim.AdamW semantics (decoupled decay, bias-corrected, eps outside sqrt)."""

    def __init__(self, lr=5e-4, betas=(0.9, 0.999), eps=1e-8, wd=0.05):
        self.lr, self.b1, self.b2, self.eps, self.wd = lr, betas[0], betas[1], eps, wd
        self.m, self.v, self.t = {}, {}, {}

    @torch.no_grad()
    def step(self, P, grads):
        for n, g in grads.items():
            if g is None:
                continue
            p = P[n]
            t = self.t.get(n, 0) + 1
            self.t[n] = t
            m = self.m.get(n, torch.zeros_like(p))
            v = self.v.get(n, torch.zeros_like(p))
            p.mul_(1 - self.lr * self.wd)
            m.mul_(self.b1).add_(g, alpha=1 - self.b1)
            v.mul_(self.b2).addcmul_(g, g, value=1 - self.b2)
            bc1 = 1 - self.b1 ** t
            bc2 = 1 - self.b2 ** t
            denom = (v.sqrt() / math.sqrt(bc2)).add_(self.eps)
            p.addcdiv_(m, denom, value=-self.lr / bc1)
            self.m[n], self.v[n] = m, v


def update_bn_buffers(bufs, trk, momentum=0.1):
    for pre, mean, var_u, updates in trk.stats:
        rm, rv = bufs[pre + ".running_mean"], bufs[pre + ".running_var"]
        for _ in range(updates):
            rm.mul_(1 - momentum).add_(mean, alpha=momentum)
            rv.mul_(1 - momentum).add_(var_u, alpha=momentum)
            bufs[pre + ".num_batches_tracked"] += 1


def train_step(P, bufs, opt, clip, mask, cfg, acts=None):
    """One train_one_epoch iteration (train_ssl_mae.py:66-89) given the mask.
    Returns (loss, grads dict)."""
    leaves = {n: p.detach().requires_grad_(p.dtype.is_floating_point) for n, p in P.items()}
    trk = _BNTracker()
    target = patchify(clip, 8)
    if cfg["ssl"]["norm_pix_loss"]:
        target = norm_pix(target)
    pred = mae_forward(leaves, clip, mask, cfg, trk, acts)
    loss = masked_mse(pred, target, mask)
    used = {n: t for n, t in leaves.items() if ".stages.3." not in n}
    gl = torch.autograd.grad(loss, list(used.values()), allow_unused=True)
    grads = dict(zip(used.keys(), gl))
    for n in leaves:
        grads.setdefault(n, None)
    if opt is not None:
        opt.step(P, grads)
    if bufs is not None:
        update_bn_buffers(bufs, trk)
    return loss.detach(), grads


def init_buffers(P):
    bufs = {}
    for n, p in P.items():
        if n.endswith(".bn.weight"):
            pre = n[: -len(".weight")]
            bufs[pre + ".running_mean"] = torch.zeros_like(p)
            bufs[pre + ".running_var"] = torch.ones_like(p)
            bufs[pre + ".num_batches_tracked"] = torch.zeros((), dtype=torch.int64)
    return bufs
