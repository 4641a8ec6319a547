"""TinyVideoMAE (reference: src/models/mae_vit_adapter.py), MI355X-native.

Same constructor (`TinyVideoMAE(encoder, config)` reading dataset.clip_len,
dataset.image_size, model.decoder_{embed_dim,num_heads,depth}), same parameter
tree and initialisation (trunc_normal pos-embeds / mask token, xavier Linear,
unit LayerNorm — mae_vit_adapter.py:57-73), same forward contract:
forward(x [B,3,T,H,W] fp32, mask bool [B,T,L]) -> pred [B, T*L, 192].

Runs on the fused HIP Functions; bf16 mode is selected by an enclosing
torch.autocast('cuda', dtype=torch.bfloat16), exactly where the reference's
train_one_epoch (train_ssl_mae.py:79) runs its forward; otherwise fp32.
"""
import torch
import torch.nn as nn

from .functions import BlockFn, EncToDecFn, HeadFn, Mode
from .optim import FlatParams


def _trunc_normal_(t, std=0.02):
    # timm.layers.trunc_normal_(tensor, mean=0, std, a=-2, b=2) (absolute bounds)
    return nn.init.trunc_normal_(t, 0.0, std, -2.0, 2.0)


def next_seed_base(root):
    """Fresh RNG base per forward: the device generator's seed (set_seed seeds it)
    plus a per-model forward counter.  The host generator — which drives the tube
    mask exactly as in the reference — is not consumed."""
    cnt = getattr(root, "_sm_fwd_count", 0)
    root._sm_fwd_count = cnt + 1
    dev = torch.cuda.current_device()
    base = torch.cuda.default_generators[dev].initial_seed()
    from .functions import splitmix64
    return splitmix64((base << 20) ^ cnt)


def make_flat(root: nn.Module, dev):
    """Lay every parameter of `root` into one flat buffer on `dev` (see optim.FlatParams)."""
    named = [(n, p) for n, p in root.named_parameters()]
    mae = getattr(root, "_mae", False)
    is_used = [not (mae and ".stages.3." in "." + n) for n, _ in named]
    used = [np for np, u in zip(named, is_used) if u]
    unused = [np for np, u in zip(named, is_used) if not u]
    flat = FlatParams(gradient_order(used) + unused, dev, n_attach=len(used))
    root._sm_flat = flat
    return flat


def ensure_flat(root: nn.Module, mode: Mode):
    """Move every parameter of `root` into one flat device buffer (once), then
    mark the start of a forward (zero-on-first-backward, bf16 shadow refresh)."""
    params = list(root.parameters())
    dev = params[0].device
    if dev.type != "cuda":
        raise RuntimeError("ssl_mae_amd models run on the GPU only (move the model with .to('cuda'))")
    # a sub-module (e.g. the MAE's encoder run on its own) uses its parent's buffer
    flat = getattr(params[0], "_sm_flat", None)
    if flat is None or flat.device != dev or any(getattr(p, "_sm_flat", None) is not flat for p in params):
        flat = make_flat(root, dev)
    flat.begin_forward(mode.bf16)
    return flat


def gradient_order(named_used):
    """The order the backward produces gradients in: reverse forward order, except
    that the MAE's own parameters (mask_token, temporal/spatial pos-embed) get their
    gradients from EncToDecFn together with enc_to_dec, not after the encoder.  The
    flat buffer follows it, so data-parallel buckets fill front to back."""
    order = list(reversed(named_used))
    own = [np for np in order if "." not in np[0]]
    rest = [np for np in order if "." in np[0]]
    at = max((i + 1 for i, (n, _) in enumerate(rest) if n.startswith("enc_to_dec.")), default=len(rest))
    return rest[:at] + own + rest[at:]


class _St:
    def __init__(self, **kw):
        self.__dict__.update(kw)


class TinyVideoMAE(nn.Module):
    def __init__(self, encoder, config):
        super().__init__()
        self.encoder = encoder
        self.clip_len = config["dataset"]["clip_len"]
        self.img_size = config["dataset"]["image_size"]
        self.patch_size = 8
        self.num_patches = (self.img_size // self.patch_size) ** 2
        self.encoder_dim = 384
        self.decoder_embed_dim = config["model"]["decoder_embed_dim"]
        self.decoder_num_heads = config["model"]["decoder_num_heads"]
        self.decoder_depth = config["model"]["decoder_depth"]
        self.enc_to_dec = nn.Linear(self.encoder_dim, self.decoder_embed_dim, bias=True)
        self.mask_token = nn.Parameter(torch.zeros(1, 1, self.decoder_embed_dim))
        self.temporal_pos_embed = nn.Parameter(torch.zeros(1, self.clip_len, 1, self.decoder_embed_dim))
        self.spatial_pos_embed = nn.Parameter(torch.zeros(1, 1, self.num_patches, self.decoder_embed_dim))
        layer = nn.TransformerEncoderLayer(d_model=self.decoder_embed_dim, nhead=self.decoder_num_heads,
                                           dim_feedforward=int(self.decoder_embed_dim * 4), batch_first=True,
                                           norm_first=True, activation="gelu")
        self.decoder_blocks = nn.TransformerEncoder(layer, num_layers=self.decoder_depth,
                                                    enable_nested_tensor=False)
        self.decoder_norm = nn.LayerNorm(self.decoder_embed_dim)
        self.decoder_pred = nn.Linear(self.decoder_embed_dim, self.patch_size ** 2 * 3, bias=True)
        self._mae = True
        encoder._sm_dec_depth = self.decoder_depth
        self.initialize_weights()
        from .tiny_vit import index_modules
        index_modules(self)

    def initialize_weights(self):
        _trunc_normal_(self.temporal_pos_embed, std=0.02)
        _trunc_normal_(self.spatial_pos_embed, std=0.02)
        _trunc_normal_(self.mask_token, std=0.02)
        self.apply(self._init_weights)

    def _init_weights(self, m):
        if isinstance(m, nn.Linear):
            nn.init.xavier_uniform_(m.weight)
            if m.bias is not None:
                nn.init.constant_(m.bias, 0)
        elif isinstance(m, nn.LayerNorm):
            nn.init.constant_(m.bias, 0)
            nn.init.constant_(m.weight, 1.0)

    def forward(self, x, mask):
        """x [B,3,T,H,W] fp32, mask bool [B,T,L] (True = masked) -> pred [B, T*L, 192]."""
        B, C, T, H, W = x.shape
        mode = Mode(torch.is_autocast_enabled("cuda"), next_seed_base(self))
        ensure_flat(self, mode)
        dev = self.mask_token.device
        if x.device != dev:
            x = x.to(dev, non_blocking=True)
        if x.dtype != torch.float32:
            x = x.float()
        m8 = mask.view(torch.uint8) if mask.dtype == torch.bool else mask.to(torch.uint8)
        if m8.device != dev:
            m8 = m8.to(dev, non_blocking=True)
        m8 = m8.reshape(B, T, -1).contiguous()
        L = m8.shape[-1]
        D = self.decoder_embed_dim
        lat = self.encoder.tokens_stage3(x, mode)                      # [B*T, H/8, W/8, 384]
        if lat.shape[1] * lat.shape[2] != L:
            raise ValueError(f"mask has {L} patches per frame, encoder produced {lat.shape[1] * lat.shape[2]}")
        lat = lat.reshape(B * T * L, self.encoder_dim)
        st = _St(mode=mode, B=B, T=T, L=L, D=D)
        xd = EncToDecFn.apply(lat, m8, st, self.enc_to_dec.weight, self.enc_to_dec.bias,
                              self.temporal_pos_embed, self.spatial_pos_embed, self.mask_token)
        for layer in self.decoder_blocks.layers:
            sa = layer.self_attn
            tr = self.training
            idx = getattr(layer, "_sm_index", 0)
            bst = _St(mode=mode, N=B, L=T * L, heads=self.decoder_num_heads, head_dim=D // self.decoder_num_heads,
                      eps=layer.norm1.eps,
                      attn_drop=sa.dropout if tr else 0.0, seed_attn=mode.seed(idx, 0),
                      drop1=layer.dropout1.p if tr else 0.0, seed1=mode.seed(idx, 1),
                      drop_ff=layer.dropout.p if tr else 0.0, seed_ff=mode.seed(idx, 2),
                      drop2=layer.dropout2.p if tr else 0.0, seed2=mode.seed(idx, 3), dp1=None, dp2=None)
            xd = BlockFn.apply(xd, bst, layer.norm1.weight, layer.norm1.bias, sa.in_proj_weight, sa.in_proj_bias,
                               sa.out_proj.weight, sa.out_proj.bias, layer.norm2.weight, layer.norm2.bias,
                               layer.linear1.weight, layer.linear1.bias, layer.linear2.weight,
                               layer.linear2.bias)
        pred = HeadFn.apply(xd, _St(mode=mode), self.decoder_norm.weight, self.decoder_norm.bias,
                            self.decoder_pred.weight, self.decoder_pred.bias)
        return pred.view(B, T * L, self.patch_size ** 2 * 3)
