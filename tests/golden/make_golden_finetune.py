"""Golden fixtures for the frozen-encoder fine-tune (BASELINE config 4) by RUNNING
the reference's TinyViT (src/models/tiny_vit.py) in the build container.

The reference's VideoClassifier (src/train_finetune.py:19-40) wraps MobileViT;
config C4 puts the MAE's TinyViT encoder in its place.  This script builds that
classifier from reference parts: `tiny_vit_21m_variant(img_size=112)` as the
backbone run through `TinyViT.forward` (all four stages, tiny_vit.py:178-186),
the MobileViT backbone's embedding rule (adaptive_avg_pool2d(feat, 1), mobilevit.py:
164-165), and VideoClassifier.forward's per-frame loop, temporal mean and Linear,
restated line for line.  Weights: the portable rule (ssl_mae_amd.init_rule) on the
whole classifier.  Parity mode: DropPath p = 0 (BN in train mode).

Sequence recorded (B=2 clips, T=16 frames, 112x112, 101 classes):
  1. linear-probe step (train_finetune.py:84-124 with mode linear_probe,
     :294-296,309-311): model.train(), backbone frozen, CE loss, AdamW on the head
     -> loss, logits, head grads, head params after the step, BN running stats
     (updated once per frame call: num_batches_tracked = T);
  2. evaluation forward (train_finetune.py:127-138): model.eval() under no_grad on
     a second clip -> logits, embeddings.
A second fixture, finetune_ftssl_b2_t2_s112.npz (ft_ssl mode, :198-210: backbone
trainable), records one fp32 training step's backbone gradients (B=2, T=2, 112x112,
DropPath 0, model.train()): per parameter the gradient sum, L2 norm and first 8
values, plus loss and logits -- the T per-frame backward groups summed into each
backbone gradient.
Run:  python tests/golden/make_golden_finetune.py
"""
import os
import sys

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as MG  # noqa: E402
from ssl_mae_amd.init_rule import apply_rule, synthetic_clip  # noqa: E402


class RefClassifier(nn.Module):
    def __init__(self, tiny_vit, num_classes, img_size):
        super().__init__()
        self.backbone = tiny_vit.tiny_vit_21m_variant(img_size=img_size, use_checkpoint=True)
        self.classifier = nn.Linear(576, num_classes)

    def embed(self, frames):
        feat = self.backbone(frames)                                # TinyViT.forward
        return F.adaptive_avg_pool2d(feat, 1).flatten(1)

    def forward(self, clip):
        B, C, T, H, W = clip.shape
        feats = torch.stack([self.embed(clip[:, :, t, :, :]) for t in range(T)], dim=1)
        return self.classifier(feats.mean(dim=1))


def main():
    tiny_vit = MG._import_reference()[0]
    torch.set_num_threads(8)
    B, T, S, NC = 2, 16, 112, 101
    model = RefClassifier(tiny_vit, NC, S)
    apply_rule(model)
    for m in model.modules():
        if hasattr(m, "drop_prob"):
            m.drop_prob = 0.0
    rec = {"B": B, "T": T, "S": S, "num_classes": NC}
    clip = torch.from_numpy(synthetic_clip(B, T, S, seed=4321))
    label = torch.tensor([3, 77])
    # 1) linear-probe step
    for p in model.backbone.parameters():
        p.requires_grad = False
    opt = torch.optim.AdamW([p for p in model.parameters() if p.requires_grad], lr=1e-3, weight_decay=0.01)
    model.train()
    opt.zero_grad(set_to_none=True)
    logits = model(clip)
    loss = nn.CrossEntropyLoss()(logits, label)
    loss.backward()
    rec["train_logits"] = logits.detach().numpy()
    rec["train_loss"] = np.float64(loss.item())
    rec["head_grad_w"] = model.classifier.weight.grad.numpy().copy()
    rec["head_grad_b"] = model.classifier.bias.grad.numpy().copy()
    opt.step()
    rec["head_w_after"] = model.classifier.weight.detach().numpy().copy()
    rec["head_b_after"] = model.classifier.bias.detach().numpy().copy()
    for n, b in model.backbone.named_buffers():
        rec["buf/" + n] = b.detach().numpy().copy()
    # 2) evaluation forward (running statistics)
    clip2 = torch.from_numpy(synthetic_clip(B, T, S, seed=8765))
    model.eval()
    with torch.no_grad():
        frames = clip2.permute(0, 2, 1, 3, 4).reshape(B * T, 3, S, S)
        feat = model.backbone(frames)
        emb = F.adaptive_avg_pool2d(feat, 1).flatten(1)
        logits2 = model(clip2)
    rec["eval_feat_shape"] = np.array(feat.shape)
    rec["eval_feat_sum"] = np.float64(feat.double().sum())
    rec["eval_feat_sumsq"] = np.float64((feat.double() ** 2).sum())
    rec["eval_emb"] = emb.numpy()
    rec["eval_logits"] = logits2.numpy()
    out = os.path.join(HERE, "finetune_b2_t16_s112.npz")
    np.savez_compressed(out, **rec)
    print(f"wrote {out}: train loss {loss.item():.6f}, eval logits[0,:3] {logits2[0, :3].tolist()}")


def ftssl_case():
    tiny_vit = MG._import_reference()[0]
    torch.set_num_threads(8)
    B, T, S, NC = 2, 2, 112, 11
    model = RefClassifier(tiny_vit, NC, S)
    apply_rule(model)
    for m in model.modules():
        if hasattr(m, "drop_prob"):
            m.drop_prob = 0.0
    clip = torch.from_numpy(synthetic_clip(B, T, S, seed=2468))
    label = torch.tensor([1, 7])
    model.train()
    logits = model(clip)
    loss = nn.CrossEntropyLoss()(logits, label)
    loss.backward()
    rec = {"B": B, "T": T, "S": S, "num_classes": NC, "loss": np.float64(loss.item()),
           "logits": logits.detach().numpy()}
    names = []
    for n, p in model.named_parameters():
        if p.grad is None:
            continue
        g = p.grad.detach().double().reshape(-1)
        names.append(n)
        rec["gsum/" + n] = np.float64(g.sum())
        rec["gl2/" + n] = np.float64(g.norm())
        rec["ghead/" + n] = g[:8].numpy().copy()
    rec["names"] = np.array(names)
    out = os.path.join(HERE, "finetune_ftssl_b2_t2_s112.npz")
    np.savez_compressed(out, **rec)
    print(f"wrote {out}: loss {loss.item():.6f}, {len(names)} parameters with gradients")


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "ftssl":
        ftssl_case()
    else:
        main()
