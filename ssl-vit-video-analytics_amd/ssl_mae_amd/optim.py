"""Flat parameter storage, fused AdamW and a GradScaler-compatible shim.

Layout in HBM: every trainable parameter of the model lives in ONE fp32 buffer
(16-byte aligned slots, ordered in reverse forward order so that gradients are
produced front-to-back during the backward — the order the data-parallel
all-reduce buckets are filled in), with a matching fp32 gradient buffer and a
bf16 shadow used as the GEMM operand in bf16 mode.  Parameters become views of
the flat buffer (state_dict keys and shapes unchanged); `p.grad` is a view of the
flat gradient buffer, which the backward kernels write directly.

AdamW follows torch.optim.AdamW (train_ssl_mae.py:163: lr from the config,
weight_decay 0.05, betas (0.9, 0.999), eps 1e-8; parameters that received no
gradient this step are skipped, as torch skips grad-None params).  The non-finite
gradient check reproduces GradScaler.step's skip (train_ssl_mae.py:87-89) without
a host sync.
"""
import torch

from . import ops as K    # every kernel launch through the torch.ops.ssl_mae dispatcher

ALIGN = 8  # elements: keeps every bf16 view 16-byte aligned


class FlatParams:
    def __init__(self, named_params, device, n_attach=None):
        self.n_attach = len(named_params) if n_attach is None else n_attach
        self.names = [n for n, _ in named_params]
        self.params = [p for _, p in named_params]
        self.offsets = []
        off = 0
        for p in self.params:
            self.offsets.append(off)
            off += (p.numel() + ALIGN - 1) // ALIGN * ALIGN
        self.total = off
        self.device = device
        self.data = torch.zeros(off, dtype=torch.float32, device=device)
        self.grad = torch.zeros(off, dtype=torch.float32, device=device)
        self.shadow = torch.zeros(off, dtype=torch.bfloat16, device=device)
        for i, (p, o) in enumerate(zip(self.params, self.offsets)):
            n = p.numel()
            self.data[o:o + n].copy_(p.data.reshape(-1).to(device))
            p.data = self.data[o:o + n].view(p.shape)
            p._sm_grad = self.grad[o:o + n].view(p.shape)
            p._sm_bf16 = self.shadow[o:o + n].view(p.shape)
            p._sm_flat = self
            p.grad = p._sm_grad if i < self.n_attach and p.requires_grad else None
        # [0, used_end): parameters on the MAE path (stage-4 params are never used by
        # forward_stage3 and, as with the reference's grad-None, are never updated)
        self.used_end = self.offsets[self.n_attach - 1] + (self.params[self.n_attach - 1].numel() + ALIGN - 1) \
            // ALIGN * ALIGN if self.n_attach else 0
        self.index = {id(p): i for i, p in enumerate(self.params)}
        self.touched = set()
        self.fresh = False
        self.shadow_dtype_ready = False
        # gradient buckets (data parallel): contiguous runs of whole parameters over
        # [0, used_end); `done()` counts finished parameters per bucket and calls the
        # ready hooks with a bucket's index as soon as its last parameter is written
        self.bucket_ranges = []
        self.bucket_of = {}
        self.ready_hooks = []
        self._pending = []
        self._finished = set()

    # ---------------------------------------------------------------- buckets
    def make_buckets(self, bucket_elems):
        ranges, of = [], {}
        start = None
        for i in range(self.n_attach):
            s = self.offsets[i]
            e = s + (self.params[i].numel() + ALIGN - 1) // ALIGN * ALIGN
            if start is None:
                start = s
            of[id(self.params[i])] = len(ranges)
            if e - start >= bucket_elems or i == self.n_attach - 1:
                ranges.append((start, e))
                start = None
        self.bucket_ranges = ranges
        self.bucket_of = of
        self._reset_buckets()
        return ranges

    def _reset_buckets(self):
        counts = [0] * len(self.bucket_ranges)
        for b in self.bucket_of.values():
            counts[b] += 1
        self._pending = counts
        self._finished = set()

    def done(self, *params):
        """Called by every backward kernel group after it has launched the writes of
        its parameters' gradients (stream-ordered: the writes precede anything the
        hooks enqueue on the same stream)."""
        if not self.ready_hooks:
            return
        for p in params:
            b = self.bucket_of.get(id(p))
            if b is None:
                continue
            if id(p) in self._finished:
                # a second gradient contribution after the bucket may already be in
                # flight on the side stream: the reduced value would race the add
                raise RuntimeError(
                    f"FlatParams.done: parameter {self.names[self.index[id(p)]]} received gradient from more "
                    "than one backward group in one step while bucketed all-reduce hooks are attached; the "
                    "overlapped all-reduce supports exactly one gradient write per parameter per backward "
                    "(run modules used several times per step without OverlappedGradAllReduce, e.g. with "
                    "dist.GradAllReduce after the backward)")
            self._finished.add(id(p))
            self._pending[b] -= 1
            if self._pending[b] == 0:
                for h in self.ready_hooks:
                    h(b)

    # ---------------------------------------------------------------- per step
    def begin_forward(self, bf16):
        """Called at the top of every model forward."""
        self.fresh = True
        if bf16:
            K.cast(self.data, torch.bfloat16, out=self.shadow)

    def touch(self, *params):
        """Called by every backward kernel group before it writes gradient sinks."""
        if self.fresh:
            self.fresh = False
            K.fill_(self.grad, 0.0)
            self.touched.clear()
            self._reset_buckets()
            for p in self.params[:self.n_attach]:
                if p.requires_grad:
                    p.grad = p._sm_grad
        for p in params:
            self.touched.add(id(p))

    def zero_grad(self):
        K.fill_(self.grad, 0.0)
        self.touched.clear()

    def touched_ranges(self):
        """Coalesced [start, end) element ranges of the params that got gradients."""
        idx = sorted(self.index[i] for i in self.touched if i in self.index)
        ranges = []
        for i in idx:
            s = self.offsets[i]
            e = s + (self.params[i].numel() + ALIGN - 1) // ALIGN * ALIGN
            if ranges and ranges[-1][1] == s:
                ranges[-1][1] = e
            else:
                ranges.append([s, e])
        return ranges


def flat_of(params):
    flats = {getattr(p, "_sm_flat", None) for p in params}
    flats.discard(None)
    return flats


class FusedAdamW:
    """Drop-in for torch.optim.AdamW over parameters living in a FlatParams buffer."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2):
        self.param_list = list(params)
        self.param_groups = [{"params": self.param_list, "lr": lr, "betas": betas, "eps": eps,
                              "weight_decay": weight_decay}]
        self._state = None
        self.grad_hooks = []      # callables(flat) run before the update (e.g. DP all-reduce)

    def _init_state(self):
        flats = flat_of(self.param_list)
        if len(flats) != 1:
            raise RuntimeError("FusedAdamW: parameters are not (yet) in one flat buffer; "
                               "run a forward pass of the model first")
        flat = flats.pop()
        dev = flat.device
        self._state = {
            "flat": flat,
            "m": torch.zeros(flat.total, dtype=torch.float32, device=dev),
            "v": torch.zeros(flat.total, dtype=torch.float32, device=dev),
            "step": torch.zeros(1, dtype=torch.int64, device=dev),
            "found_inf": torch.zeros(1, dtype=torch.int32, device=dev),
        }

    @property
    def flat(self):
        if self._state is None:
            self._init_state()
        return self._state["flat"]

    def zero_grad(self, set_to_none=True):
        flats = flat_of(self.param_list)
        for f in flats:
            f.zero_grad()

    def step(self, closure=None):
        if self._state is None:
            self._init_state()
        st = self._state
        flat = st["flat"]
        for hook in self.grad_hooks:
            hook(flat)
        g = self.param_groups[0]
        b1, b2 = g["betas"]
        K.fill_(st["found_inf"].view(torch.float32), 0.0)
        ranges = flat.touched_ranges()
        for s, e in ranges:
            K.nonfinite(flat.grad[s:e], st["found_inf"])
        for i, (s, e) in enumerate(ranges):
            K.adamw(flat.data[s:e], flat.grad[s:e], st["m"][s:e], st["v"][s:e], g["lr"], b1, b2, g["eps"],
                    g["weight_decay"], st["found_inf"], st["step"], advance_step=(i == len(ranges) - 1))
        return None

    def state_dict(self):
        """torch.optim-style state: per-parameter `exp_avg` / `exp_avg_sq` keyed by the
        parameter's name in the flat buffer (layout-independent), plus the shared
        step count.  Tensors are clones (safe to torch.save while training goes on)."""
        groups = [{k: v for k, v in self.param_groups[0].items() if k != "params"}]
        st = self._state
        if st is None:
            return {"param_groups": groups, "state": {}, "step": 0}
        flat = st["flat"]
        mine = {id(p) for p in self.param_list}
        per = {}
        for name, p, off in zip(flat.names, flat.params, flat.offsets):
            if id(p) not in mine:
                continue
            n = p.numel()
            per[name] = {"exp_avg": st["m"][off:off + n].view(p.shape).clone(),
                         "exp_avg_sq": st["v"][off:off + n].view(p.shape).clone()}
        return {"param_groups": groups, "state": per, "step": int(st["step"].item())}

    def load_state_dict(self, sd):
        """Inverse of state_dict (the model must have run its flat-buffer setup, e.g.
        one forward or `ensure_flat`)."""
        if self._state is None:
            self._init_state()
        st = self._state
        flat = st["flat"]
        g = sd.get("param_groups", [{}])[0]
        for k in ("lr", "betas", "eps", "weight_decay"):
            if k in g:
                self.param_groups[0][k] = tuple(g[k]) if k == "betas" else g[k]
        by_name = dict(zip(flat.names, zip(flat.params, flat.offsets)))
        for name, s in sd.get("state", {}).items():
            if name not in by_name:
                raise KeyError(f"optimizer state for unknown parameter {name}")
            p, off = by_name[name]
            n = p.numel()
            st["m"][off:off + n].copy_(s["exp_avg"].reshape(-1).to(st["m"].device))
            st["v"][off:off + n].copy_(s["exp_avg_sq"].reshape(-1).to(st["v"].device))
        st["step"].fill_(int(sd.get("step", 0)))


class GradScaler:
    """torch.amp.GradScaler-compatible shim.  bf16 needs no loss scaling (the scale is
    a power of two, so the reference's scale/unscale is exact); the inf/nan skip is
    done inside FusedAdamW.step."""

    def __init__(self, device="cuda", enabled=True, **_):
        self.enabled = enabled

    def scale(self, loss):
        return loss

    def step(self, optimizer, *a, **k):
        return optimizer.step()

    def update(self, new_scale=None):
        pass

    def get_scale(self):
        return 1.0

    def state_dict(self):
        return {"scale": 1.0, "enabled": self.enabled}

    def load_state_dict(self, sd):
        self.enabled = bool(sd.get("enabled", self.enabled))

    def unscale_(self, optimizer):
        pass
