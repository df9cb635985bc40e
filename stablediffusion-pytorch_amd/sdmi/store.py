"""Flat fp32 parameter / gradient storage for the UNet family.

Every parameter (and its gradient) is a view into one flat fp32 buffer, ordered so that
  * the backward pass produces gradients roughly front-to-back (buckets can be all-reduced while
    the rest of the backward runs),
  * all t_emb_layers weights / biases form single contiguous runs (one GEMM covers them), and so do all
    context_proj weights / biases (one forward GEMM of the text context, one weight-gradient GEMM),
  * the optimizer is one elementwise pass over three flat buffers.
Keys are the reference's state-dict keys (models/unet_cond_base.py, models/blocks.py)."""
import re

import torch

from .unet_engine import cross_list, layout, resnet_list


def param_label(key):
    """Block label (engine tape label) whose backward finalises this parameter's gradient."""
    m = re.match(r"(downs|mids|ups)\.(\d+)\.", key)
    if ".t_emb_layers." in key and key.endswith(".weight"):
        return "time"  # one GEMM for all t_emb_layers weights, after every block
    if ".context_proj." in key:
        return "time"  # one GEMM for all context_proj weights and biases, after every block
    if m:
        return f"{m.group(1)}.{m.group(2)}"
    if key.startswith("norm_out") or key.startswith("conv_out"):
        return "head"
    if key.startswith("t_proj") or key.startswith("class_emb"):
        return "time"
    return "input"


def _tail_key(k):
    """the parameters flat_order puts last (read first by the forward): conv_in, cond_conv_in, t_proj, class_emb"""
    return not re.match(r"(downs|mids|ups)\.", k) and not k.startswith("norm_out") and not k.startswith("conv_out")


def flat_order(cfg, keys):
    L = layout(cfg)
    nd = len(L["down"]) - 1
    nm = len(L["mid"]) - 1
    res = resnet_list(L)
    tw = [f"{p}.t_emb_layers.{l}.1.weight" for (p, l, ci, co) in res]
    tb = [f"{p}.t_emb_layers.{l}.1.bias" for (p, l, ci, co) in res]
    cross = cross_list(L) if L["text"] else []
    cw = [f"{p}.context_proj.{l}.weight" for (p, l, c) in cross]
    cb = [f"{p}.context_proj.{l}.bias" for (p, l, c) in cross]
    special = set(tw) | set(tb) | set(cw) | set(cb)

    def rank(k):
        m = re.match(r"(downs|mids|ups)\.(\d+)\.", k)
        if k.startswith("norm_out") or k.startswith("conv_out"):
            return 0
        if m:
            kind, i = m.group(1), int(m.group(2))
            if kind == "ups":
                return 1 + (nd - 1 - i)
            if kind == "mids":
                return 1 + nd + (nm - 1 - i)
            return 1 + nd + nm + (nd - 1 - i)
        return 10_000  # t_proj, conv_in, cond_conv_in, class_emb: last in backward

    rest = sorted([k for k in keys if k not in special], key=lambda k: (rank(k), keys.index(k)))
    tail = [k for k in rest if rank(k) == 10_000]
    body = [k for k in rest if rank(k) != 10_000]
    return body + tw + tb + cw + cb + tail


def unet_gemm_natural(key, shape):
    """UNet conv weights kept in the GEMM-natural (co, kh, kw, ci) order in the flat buffers (FlatStore natural=):
    the resnet 3x3 convs and the stride-2 down-sampling convs, whose weight gradients the engine then writes with
    16-byte row stores (a torch-layout (co, ci, kh, kw) gradient is a stride-(kh*kw) column scatter: the 4x4-level
    3x3 weight gradient measured 38 -> 16 us, scripts/wg_anatomy.py) and whose forward packs become plain casts.
    conv_in / conv_out (padded channels) and the transposed up-sampling convs ((ci, co, kh, kw)) keep torch order."""
    return (len(shape) == 4 and shape[2] * shape[3] > 1 and key.endswith(".weight")
            and (".resnet_conv_first." in key or ".resnet_conv_second." in key or key.endswith("down_sample_conv.weight")))


class FlatStore:
    def __init__(self, shapes, cfg, device, with_grads=True, order=None, grad_tail=0, natural=None):
        """grad_tail: extra fp32 slots after the gradients (inside the all-reduced buffer, outside every parameter and
        the gradient norm): the data-parallel trainer's non-finite-loss flag rides in the last bucket.
        natural: predicate (key, shape) -> True for 4-d conv weights stored in (co, kh, kw, ci) order; their views
        (parameters, gradients, EMA, Adam moments) are torch-shaped (co, ci, kh, kw) permutations of that memory."""
        keys = list(shapes.keys())
        self.natural = {k for k in keys if natural is not None and natural(k, tuple(shapes[k]))}
        self.order = list(order) if order is not None else flat_order(cfg, keys)
        assert sorted(self.order) == sorted(keys), "flat order must cover every parameter exactly once"
        self.shapes = dict(shapes)
        self.offsets = {}
        off = 0
        for k in self.order:
            n = 1
            for s in shapes[k]:
                n *= s
            self.offsets[k] = (off, n)
            # 32-B aligned starts: 16-B vector loads of fp32 biases
            off += (n + 7) // 8 * 8
        self.numel = off
        self.params = torch.zeros(off, dtype=torch.float32, device=device)
        self.grads = torch.zeros(off + grad_tail, dtype=torch.float32, device=device) if with_grads else None
        self.p = {k: self.view(self.params, k) for k in self.order}
        self.g = {k: self.view(self.grads, k) for k in self.order} if with_grads else None

    def forward_chunks(self, n, lead=False):
        """~n contiguous ranges [lo, hi) of the flat buffer in FORWARD order (descending offsets: the backward
        finalises the last layers first, so the flat order is roughly reverse forward order), split at parameter
        starts; returns (ranges, chunk_of_key).
        lead (UNet flat_order): the runs the forward reads first become chunks of their own ahead of the n -- the
        input / time-MLP parameters, the context projections of every cross-attention, the time-embedding projections
        of every resnet, then the first two down blocks whole -- so the next forward's first kernels wait for the
        optimizer update of ~1 M parameters instead of one sixth of all of them, and every later wait is for the block
        the forward is about to run."""
        cuts, hi = [], self.numel
        if lead:
            groups = [lambda k: _tail_key(k), lambda k: ".context_proj." in k, lambda k: ".t_emb_layers." in k,
                      lambda k: k.startswith("downs.0.") and ".t_emb_layers." not in k and ".context_proj." not in k,
                      lambda k: k.startswith("downs.1.") and ".t_emb_layers." not in k and ".context_proj." not in k]
            for g in groups:
                offs = [self.offsets[k][0] for k in self.order if g(k)]
                if offs and min(offs) < hi:
                    cuts.append((min(offs), hi))
                    hi = min(offs)
        starts = sorted(off for off, _ in self.offsets.values() if off < hi)
        target = max(1, hi // n)
        for s in reversed(starts):  # walk from the top of the (remaining) buffer down
            if hi - s >= target and s > 0:
                cuts.append((s, hi))
                hi = s
        cuts.append((0, hi))
        ranges = [c for c in cuts if c[1] > c[0]]
        chunk_of = {}
        for k, (off, _) in self.offsets.items():
            chunk_of[k] = next(i for i, (lo, hi) in enumerate(ranges) if lo <= off < hi)
        return ranges, chunk_of

    def view(self, flat, k):
        off, n = self.offsets[k]
        if k in self.natural:
            co, ci, kh, kw = self.shapes[k]
            return flat[off:off + n].view(co, kh, kw, ci).permute(0, 3, 1, 2)
        return flat[off:off + n].view(self.shapes[k])

    def load(self, state_dict):
        with torch.no_grad():
            for k in self.order:
                self.p[k].copy_(state_dict[k])

    def state_dict(self):
        return {k: self.p[k] for k in self.shapes}
