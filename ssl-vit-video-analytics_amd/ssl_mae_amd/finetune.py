"""Frozen-encoder fine-tune (BASELINE config 4), MI355X-native.

Reference: src/train_finetune.py.  Its `VideoClassifier` (:19-40) runs a backbone
per frame (`_, emb = self.backbone(clip[:, :, t])`), stacks the per-frame
embeddings, averages them over time and applies one Linear; `load_pretrained_ssl`
(:43-63) loads the `encoder.*` keys of an SSL checkpoint into the backbone; the
four modes (:198-210) freeze or unfreeze the backbone; `train_one_epoch` (:84-124)
trains under `model.train()` (so BatchNorm uses batch statistics even when the
backbone is frozen) and `evaluate` (:127-153) runs under `model.eval()` + no_grad.

The reference's backbone is MobileViT-S; config C4 fine-tunes the MAE-pretrained
TinyViT encoder instead ("ViT-Tiny fine-tune with frozen HIP encoder + linear
head").  `TinyViTBackbone` is the TinyViT of tiny_vit.py (same state_dict keys as
the MAE's `encoder.`) with the MobileViT backbone's output contract
(`(feat, emb)`, emb = adaptive-avg-pooled feat, mobilevit.py:163-166), running all
four stages (`TinyViT.forward`, tiny_vit.py:178-186: stage 4 = 576-d, 18 heads of
d=32, 7x7 tokens at 112^2).

Execution (all HIP): the stem / MBConv / transformer-block kernels of the MAE path
(BatchNorm in eval mode from the running statistics, or batch statistics in train
mode), per-frame pooling and the temporal mean as `sm_segment_mean`, the head as
the bf16/fp32 GEMM.  Train mode keeps the reference's per-frame backbone calls (T
batches of B frames, so BatchNorm statistics and running-stat updates are those of
each time step); eval mode runs all B*T frames in one batch (running statistics
make frames independent) and reads them straight from the [B,3,T,H,W] clip.
"""
import os

import torch
import torch.nn as nn

from . import ops as K    # every kernel launch through the torch.ops.ssl_mae dispatcher
from .functions import Mode, splitmix64
from .mae_vit_adapter import ensure_flat, next_seed_base
from .tiny_vit import TinyViT


class SegMeanFn(torch.autograd.Function):
    """x [G*R, C] (any float dtype) -> fp32 [G, C] mean over each segment's R rows."""

    @staticmethod
    def forward(ctx, x, G, R):
        C = x.shape[-1]
        ctx.shape = (G, R, C, x.dtype)
        return K.segment_mean(x.reshape(G * R, C).contiguous(), G, R, C)

    @staticmethod
    def backward(ctx, dy):
        G, R, C, dtype = ctx.shape
        return K.segment_mean_bwd(dy.float().contiguous(), G, R, C, dtype), None, None


class HeadLinearFn(torch.autograd.Function):
    """nn.Linear on the GEMM kernel (fp32: the embeddings are fp32), gradients returned
    to autograd for the head's (torch) optimizer."""

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        return K.linear(x.contiguous(), w.detach().contiguous(), b.detach().contiguous())

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dy = dy.float().contiguous()
        dw = torch.empty(w.shape, dtype=torch.float32, device=w.device)
        K.linear_dw(dy, x, dw, accumulate=False)
        M, N = dy.shape
        ones = K.fill_(torch.empty(M, dtype=torch.float32, device=dy.device), 1.0)
        db = torch.empty(N, dtype=torch.float32, device=w.device)
        K.gemm(ones, dy, db, 1, N, M, 0, 1, M, N, N)          # db = 1^T dy (any class count)
        dx = K.linear_dx(dy, w.detach().contiguous()) if ctx.needs_input_grad[0] else None
        return dx, dw, db


class TinyViTBackbone(TinyViT):
    """TinyViT (tiny_vit_21m_variant) with the backbone contract of
    MobileViTBackbone.forward (mobilevit.py:157-166): x [N,3,H,W] -> (feat [N,576,h,w],
    emb [N,576])."""

    def embed(self, x, mode, frames=None):
        tok = self.tokens_all(x, mode)                       # [N, h, w, 576] channels-last
        N, h, w, C = tok.shape
        return SegMeanFn.apply(tok.reshape(N * h * w, C), N, h * w), tok

    def forward(self, x):
        mode = Mode(torch.is_autocast_enabled("cuda"), next_seed_base(self))
        ensure_flat(self, mode)
        emb, tok = self.embed(x, mode)
        return tok.permute(0, 3, 1, 2), emb


def tiny_vit_backbone(img_size=112, use_checkpoint=True, **kwargs):
    return TinyViTBackbone(img_size=img_size, embed_dims=[96, 192, 384, 576], depths=[2, 2, 6, 2],
                           num_heads=[3, 6, 12, 18], use_checkpoint=use_checkpoint, **kwargs)


def frame_modes(mode, T):
    """One Mode per per-frame backbone call of a train-mode forward: the same
    precision, seed bases mixed with the time index so the DropPath masks of the T
    calls are independent (the reference draws fresh masks on every backbone call).
    Each call's checkpoint recompute / backward reuses its own Mode, so replay stays
    exact."""
    return [Mode(mode.bf16, splitmix64(mode.seed_base ^ splitmix64(0x5EED0000 + t))) for t in range(T)]


class VideoClassifier(nn.Module):
    """train_finetune.py:19-40 with the MAE-pretrained TinyViT as backbone."""

    def __init__(self, num_classes, embed_dim=576, img_size=112, backbone=None):
        super().__init__()
        self.backbone = backbone if backbone is not None else tiny_vit_backbone(img_size=img_size)
        self.classifier = nn.Linear(embed_dim, num_classes)

    def forward(self, clip):
        """clip [B, C, T, H, W] -> logits [B, num_classes]."""
        B, C, T, H, W = clip.shape
        bb = self.backbone
        if clip.dtype != torch.float32:
            clip = clip.float()
        mode = Mode(torch.is_autocast_enabled("cuda"), next_seed_base(bb))
        ensure_flat(bb, mode)
        if bb.training:
            # per-frame backbone calls as the reference (BatchNorm batch statistics and
            # running-stat updates per time step); each call draws its own DropPath masks
            # (the reference's per-call torch RNG draws), so each gets its own seed base
            feats = torch.stack([bb.embed(clip[:, :, t], m)[0] for t, m in enumerate(frame_modes(mode, T))],
                                dim=1)   # [B, T, D]
        else:
            feats = bb.embed(clip, mode)[0].view(B, T, -1)       # frames b*T + t, one batch
        video_emb = SegMeanFn.apply(feats.reshape(B * T, -1), B, T)
        return HeadLinearFn.apply(video_emb, self.classifier.weight, self.classifier.bias)


def load_pretrained_ssl(model, ckpt_path):
    """train_finetune.py:43-63, plus the checkpoint bridge the reference lacks: the
    MAE driver writes the encoder WITHOUT the `encoder.` prefix
    (train_ssl_mae.py:190-194, `encoder_ep{N}.pth`), which the reference's loader
    silently skips; such a file is loaded as the backbone state directly.  A full
    MAE state (`encoder.`-prefixed, optionally under "model") loads as in the
    reference."""
    if ckpt_path is None or not os.path.isfile(ckpt_path):
        print("[INFO] No SSL checkpoint loaded")
        return False
    ckpt = torch.load(ckpt_path, map_location="cpu", weights_only=True)
    state = ckpt.get("model", ckpt)
    backbone_state = {k[len("encoder."):]: v for k, v in state.items() if k.startswith("encoder.")}
    if not backbone_state:
        own = set(model.backbone.state_dict())
        backbone_state = {k: v for k, v in state.items() if k in own}
    missing, unexpected = model.backbone.load_state_dict(backbone_state, strict=False)
    print(f"[INFO] Loaded SSL backbone weights from {ckpt_path}")
    if missing:
        print(f"[INFO] Missing keys: {len(missing)}")
    if unexpected:
        print(f"[INFO] Unexpected keys: {len(unexpected)}")
    return True


def set_requires_grad(module, flag):
    for p in module.parameters():
        p.requires_grad = flag


def accuracy_topk(logits, targets, topk=(1,)):
    """train_finetune.py:71-81."""
    maxk = max(topk)
    _, pred = logits.topk(maxk, dim=1, largest=True, sorted=True)
    correct = pred.t().eq(targets.view(1, -1))
    return {k: (correct[:k].reshape(-1).float().sum(0) / targets.size(0)).item() for k in topk}


def train_one_epoch(model, loader, optimizer, scaler, device, cfg, log_f):
    """train_finetune.py:84-124 (bf16 autocast: the HIP kernels' reduced precision)."""
    import time
    model.train()
    ce_loss = nn.CrossEntropyLoss()
    total_loss = 0.0
    t0 = time.time()
    for step, (clip, label) in enumerate(loader):
        clip = clip.to(device, non_blocking=True)
        label = label.to(device, non_blocking=True)
        optimizer.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=bool(cfg["training"]["amp"])):
            logits = model(clip)
        loss = ce_loss(logits.float(), label)
        if scaler is not None:
            scaler.scale(loss).backward()
            scaler.step(optimizer)
            scaler.update()
        else:
            loss.backward()
            optimizer.step()
        total_loss += loss.item()
        if (step + 1) % cfg["training"]["log_interval"] == 0:
            msg = f"[INFO] step={step + 1}/{len(loader)} loss={loss.item():.4f}"
            print(msg)
            log_f.write(msg + "\n")
            log_f.flush()
    avg_loss = total_loss / max(1, len(loader))
    msg = f"[INFO] Epoch train finished, avg_loss={avg_loss:.4f}, time={time.time() - t0:.1f}s"
    print(msg)
    log_f.write(msg + "\n")
    log_f.flush()
    return avg_loss


@torch.no_grad()
def evaluate(model, loader, device, topk, log_f, split="val"):
    """train_finetune.py:127-153."""
    model.eval()
    total = 0
    correct = {k: 0.0 for k in topk}
    for clip, label in loader:
        clip = clip.to(device, non_blocking=True)
        label = label.to(device, non_blocking=True)
        acc = accuracy_topk(model(clip), label, topk=topk)
        bs = label.size(0)
        total += bs
        for k in topk:
            correct[k] += acc[k] * bs
    msg = f"[INFO] {split} results: " + ", ".join(f"Top-{k}: {correct[k] / total:.4f}" for k in topk)
    print(msg)
    log_f.write(msg + "\n")
    log_f.flush()
    return {k: correct[k] / total for k in topk}


def resolve_mode(ft_cfg, cli_mode):
    """train_finetune.py:198-210."""
    mode = cli_mode or ft_cfg.get("experiment", {}).get("mode", "ft_ssl")
    valid = {"ft_random", "linear_probe", "ft_ssl", "two_stage"}
    if mode not in valid:
        raise ValueError(f"[ERROR] Unknown mode={mode}, must be one of {sorted(list(valid))}")
    return mode


def build_optimizer(ft_cfg, model, mode):
    """train_finetune.py:164-195 (torch.optim.AdamW over the trainable parameters;
    the backbone's parameters are views of its flat buffer, their .grad views of the
    flat gradient buffer the HIP backward writes)."""
    wd = float(ft_cfg["training"]["weight_decay"])
    if mode == "two_stage":
        tr = ft_cfg["training"]
        head_lr = float(tr.get("head_lr", tr["learning_rate"]))
        backbone_lr = float(tr.get("backbone_lr", tr["learning_rate"]))
        groups = [{"params": list(model.classifier.parameters()), "lr": head_lr, "weight_decay": wd}]
        bb = [p for p in model.backbone.parameters() if p.requires_grad]
        if bb:
            groups.append({"params": bb, "lr": backbone_lr, "weight_decay": wd})
        return torch.optim.AdamW(groups)
    return torch.optim.AdamW([p for p in model.parameters() if p.requires_grad],
                             lr=float(ft_cfg["training"]["learning_rate"]), weight_decay=wd)
