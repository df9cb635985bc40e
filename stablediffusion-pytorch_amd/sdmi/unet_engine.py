"""Explicit forward/backward schedule of the reference UNet family on the HIP kernels of libsdmi.so.

Mirrors models/unet_cond_base.py:124-183 (cond) and models/unet_base.py:68-100 (uncond) with the
blocks of models/blocks.py (DownBlock :27-146, MidBlock :149-267, UpBlockUnet :373-499), re-planned
for MI355X:
  * activations are NHWC bf16 2-D views [pixels, C] (row stride = ld), so every 1x1 conv and
    attention projection is a plain GEMM and channel concatenation is free: a skip tensor is
    produced straight into the upper half of its concat buffer;
  * each conv is one implicit-GEMM launch (fwd / dgrad / wgrad), stride-2 transposed convs and
    stride-2 conv gradients are four sub-pixel 2x2 GEMMs;
  * epilogues fuse bias, the per-(batch, channel) time-embedding bias and residual adds;
  * all t_emb_layers of the network are one GEMM (their weights and gradients are contiguous);
  * GroupNorm(+SiLU) statistics/apply/backward and attention are the dedicated kernels;
  * the backward pass is an explicit reverse schedule (a tape), gradients of activations flow in
    place through residual paths, parameter gradients are written once into caller-owned fp32
    views (a flat buffer in the trainer), so no autograd graph or aten kernel runs per op.
Parameters are referenced by the reference's state-dict keys.
"""
import contextlib
import os

import torch

from . import _lib
from . import kernels as K
from . import plan
from . import streams

# GroupNorm-backward statistics from the producing data-gradient GEMM: used where a sample has >= GN_FUSE_MIN_P pixels
# (the 32^2 level of the CelebHQ latents). Same-box A/B of the cond-UNet step (scripts/gpu_bisect.sh): every level
# 13.94 / 13.90, P >= 1024 13.89 / 13.89, none 13.98 / 13.99 ms -- at 16^2 and below the statistics epilogue and the
# statistics reducer cost more than the standalone single-pass GroupNorm they replace.
GN_FUSE_MIN_P = 1024


def _gn_req(x, tab, P, C, silu):
    return K.gn_request(x, tab, P, C, silu) if P >= GN_FUSE_MIN_P else None


def layout(cfg):
    down = list(cfg["down_channels"])
    mid = list(cfg["mid_channels"])
    cond = cfg.get("condition_config") or {}
    types = cond.get("condition_types", []) if cond else []
    L = dict(text="text" in types, image="image" in types, klass="class" in types,
             G=cfg["norm_channels"], heads=cfg["num_heads"], T=cfg["time_emb_dim"],
             n_down=cfg["num_down_layers"], n_mid=cfg["num_mid_layers"], n_up=cfg["num_up_layers"],
             conv_out=cfg["conv_out_channels"], down=down, mid=mid,
             down_sample=list(cfg["down_sample"]), attn=list(cfg["attn_down"]))
    if L["text"]:
        L["ctx_dim"] = cond["text_condition_config"]["text_embed_dim"]
    if L["image"]:
        ic = cond["image_condition_config"]
        L["im_in"] = ic["image_condition_input_channels"]
        L["im_out"] = ic["image_condition_output_channels"]
    if L["klass"]:
        L["num_classes"] = cond["class_condition_config"]["num_classes"]
    return L


def resnet_list(L):
    """(prefix, index, cin, cout) of every resnet in forward order (its t_emb_layers share one GEMM)."""
    out = []
    nd = len(L["down"]) - 1
    for i in range(nd):
        for l in range(L["n_down"]):
            out.append((f"downs.{i}", l, L["down"][i] if l == 0 else L["down"][i + 1], L["down"][i + 1]))
    for i in range(len(L["mid"]) - 1):
        for l in range(L["n_mid"] + 1):
            out.append((f"mids.{i}", l, L["mid"][i] if l == 0 else L["mid"][i + 1], L["mid"][i + 1]))
    for j, i in enumerate(reversed(range(nd))):
        cin = L["down"][i] * 2
        cout = L["down"][i - 1] if i != 0 else L["conv_out"]
        for l in range(L["n_up"]):
            out.append((f"ups.{j}", l, cin if l == 0 else cout, cout))
    return out


def cross_list(L):
    """(block prefix, layer, channels) of every cross-attention, in forward order."""
    nd = len(L["down"]) - 1
    out = []
    for i in range(nd):
        out += [(f"downs.{i}", l, L["down"][i + 1]) for l in range(L["n_down"])]
    for i in range(len(L["mid"]) - 1):
        out += [(f"mids.{i}", l, L["mid"][i + 1]) for l in range(L["n_mid"])]
    for j, i in enumerate(reversed(range(nd))):
        cout = L["down"][i - 1] if i != 0 else L["conv_out"]
        out += [(f"ups.{j}", l, cout) for l in range(L["n_up"])]
    return out


class PackPlan:
    """bf16 GEMM-layout copies of the fp32 weights, refreshed by one batched pack launch."""

    def __init__(self, device):
        self.device = device
        self.items = []  # (name, src tensor, dims, shape of packed view)
        self.titems = []  # layouts derived from packed views by per-tap transposes (add_transpose)
        self.total = 0
        self.views = {}

    def add(self, name, src, O, I, Ipad, KH, KW, so, si, skh, skw, kh_off=0, kh_mul=1, kw_off=0, kw_mul=1,
            rows=None, into=None, row0=0, col0=0):
        """Pack dst[o][a][b][i] = src[o*so + i*si + (kh_off+kh_mul*a)*skh + (kw_off+kw_mul*b)*skw]
        (into a reserved matrix at row row0 / column col0 when `into` is given)."""
        n = (rows or O) * KH * KW * Ipad
        dst_ld = 0
        assert Ipad % 8 == 0, "pack_kernel writes 8 bf16 (16 bytes) per thread"
        assert KH * KW * (Ipad + 8) <= 16384, "pack_kernel stages one destination row in 32 KiB of LDS"
        if into is None:
            off = self.total
            self.total += (n + 63) // 64 * 64
            self.views[name] = (off, (rows or O), KH * KW * Ipad)
            dst_off = off
        else:
            base, _, width = self.views[into]
            dst_off = base + row0 * width + col0
            dst_ld = width if width != KH * KW * Ipad else 0
            assert width % 8 == 0 and (row0 * width + col0) % 8 == 0, "16-byte aligned pack destination"
        self.items.append(dict(src=src, dst_off=dst_off, O=O, I=I, Ipad=Ipad, KH=KH, KW=KW, so=so, si=si, skh=skh,
                               skw=skw, kh_off=kh_off, kh_mul=kh_mul, kw_off=kw_off, kw_mul=kw_mul, dst_ld=dst_ld))

    def add_transpose(self, name, src_view, O, I, taps, smap, src_tap, src_col0=0, rows=None, opad=None):
        """Derived layout from an already-packed view (run after the packs, bf16 -> bf16, per-tap transpose):
        name[i][t][o] = src_view[o][src_col0 + smap[t] * src_tap + i] for o < O, i < I; the view is
        [rows or I][taps * (opad or O)] (padding rows / columns stay zero)."""
        Opad = opad or O
        assert Opad % 8 == 0 and src_tap % 8 == 0 and src_col0 % 8 == 0 and len(smap) == taps <= 16
        width = taps * Opad
        off = self.total
        self.total += ((rows or I) * width + 63) // 64 * 64
        self.views[name] = (off, rows or I, width)
        # data-gradient layouts (#d, #t) are read only by the backward: packed after every forward chunk
        self.titems.append(dict(dst_off=off, src_view=src_view, src_col0=src_col0, O=O, I=I, taps=taps,
                                smap=list(smap), src_tap=src_tap, dst_ld=width, dst_tap=Opad, late="#f" not in name))

    def reserve(self, name, rows, width):
        off = self.total
        self.total += (rows * width + 63) // 64 * 64
        self.views[name] = (off, rows, width)

    def set_chunks(self, chunk_of_ptr, n):
        """Split the packing into per-chunk launches: chunk_of_ptr(data_ptr) -> chunk index (< n) of a source
        parameter. run_chunk(c) then packs only the views whose sources lie in chunk c (derived views after their
        source) and run_chunk(late_chunk) the backward-only derived views; view_chunk[name] is the chunk after
        which a packed view is complete."""
        self.chunk_of_ptr = chunk_of_ptr
        self.n_declared = n
        self.finalize()

    def finalize(self):
        self.buf = torch.zeros(max(self.total, 64), dtype=torch.bfloat16, device=self.device)
        chunk = _lib.lib().sdmi_pack_chunk()
        cof = getattr(self, "chunk_of_ptr", None)
        item_chunk = [cof(it["src"].data_ptr()) if cof else 0 for it in self.items]
        starts = sorted((off, name) for name, (off, rows, width) in self.views.items())
        self.view_chunk = {}

        def view_of(dst_off):
            name = None
            for off, nm in starts:
                if off > dst_off:
                    break
                name = nm
            return name

        for j, it in enumerate(self.items):  # a view is complete after the latest chunk of the items writing it
            nm = view_of(it["dst_off"])
            self.view_chunk[nm] = max(self.view_chunk.get(nm, 0), item_chunk[j])
        titem_chunk = []
        for it in self.titems:  # a derived view is produced right after its source view
            c = self.view_chunk.get(it["src_view"], 0)
            titem_chunk.append(c)
            self.view_chunk[view_of(it["dst_off"])] = c
        nreg = max(item_chunk + titem_chunk + [getattr(self, "n_declared", 1) - 1]) + 1
        self.late_chunk = None
        if any(it["late"] for it in self.titems):
            self.late_chunk = nreg
            for j, it in enumerate(self.titems):
                if it["late"]:
                    assert self.view_chunk[it["src_view"]] < nreg
                    titem_chunk[j] = nreg
                    self.view_chunk[view_of(it["dst_off"])] = nreg
        late_views = {view_of(it["dst_off"]) for it in self.titems if it["late"]}
        assert not any(not it["late"] and it["src_view"] in late_views for it in self.titems), \
            "a forward view derived from a backward-only view"
        self.nchunks = nreg + (self.late_chunk is not None)
        descs = (_lib.PackDesc * len(self.items))()
        bmaps = [[] for _ in range(self.nchunks)]
        for j, it in enumerate(self.items):
            d = descs[j]
            d.src = it["src"].data_ptr()
            d.dst = self.buf.data_ptr() + 2 * it["dst_off"]
            d.so, d.si, d.skh, d.skw = it["so"], it["si"], it["skh"], it["skw"]
            for f in ("O", "I", "Ipad", "KH", "KW", "kh_off", "kh_mul", "kw_off", "kw_mul", "dst_ld"):
                setattr(d, f, it[f])
            row = it["KH"] * it["KW"] * it["Ipad"]
            bmaps[item_chunk[j]] += [(j, o) for o in range(0, it["O"], max(1, chunk // row))]
        raw = bytes(descs)
        self.desc_dev = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(self.device)
        self.bmap_dev = [torch.tensor(b or [(0, 0)], dtype=torch.int32).reshape(-1).to(self.device) for b in bmaps]
        self.nblocks = [len(b) for b in bmaps]
        self.ptrs = [it["src"].data_ptr() for it in self.items]
        tdescs = (_lib.TPackDesc * max(1, len(self.titems)))()
        tmaps = [[] for _ in range(self.nchunks)]
        for j, it in enumerate(self.titems):
            d = tdescs[j]
            sbase, _, swidth = self.views[it["src_view"]]
            d.src = self.buf.data_ptr() + 2 * (sbase + it["src_col0"])
            d.dst = self.buf.data_ptr() + 2 * it["dst_off"]
            d.O, d.I, d.taps = it["O"], it["I"], it["taps"]
            d.src_ld, d.src_tap, d.dst_ld, d.dst_tap = swidth, it["src_tap"], it["dst_ld"], it["dst_tap"]
            assert swidth % 8 == 0
            for t, v in enumerate(it["smap"]):
                d.smap[t] = v
            tmaps[titem_chunk[j]] += [(j, i, o, t) for i in range(0, it["I"], 64) for o in range(0, it["O"], 64)
                                      for t in range(it["taps"])]
        self.tdesc_dev = torch.frombuffer(bytearray(bytes(tdescs)), dtype=torch.uint8).to(self.device)
        self.tmap_dev = [torch.tensor(m or [(0, 0, 0, 0)], dtype=torch.int32).reshape(-1).to(self.device)
                         for m in tmaps]
        self.ntiles = [len(m) for m in tmaps]

    def view(self, name):
        off, rows, width = self.views[name]
        return self.buf[off:off + rows * width].view(rows, width)

    def run(self):
        """Refresh every packed view."""
        for c in range(self.nchunks):
            self.run_chunk(c)

    def run_chunk(self, c):
        """Pack the views of chunk c (no-op for a chunk without views)."""
        _lib.check(_lib.lib().sdmi_pack_weights(self.desc_dev.data_ptr(), self.bmap_dev[c].data_ptr(), self.nblocks[c],
                                                K._stream()), "sdmi_pack_weights")
        _lib.check(_lib.lib().sdmi_pack_transpose(self.tdesc_dev.data_ptr(), self.tmap_dev[c].data_ptr(),
                                                  self.ntiles[c], K._stream()), "sdmi_pack_transpose")

    def stale(self):
        return any(it["src"].data_ptr() != p for it, p in zip(self.items, self.ptrs))


class Grads:
    """Activation-gradient buffers; names that share storage (concat halves) share one buffer."""

    def __init__(self, device):
        self.device = device
        self.groups = {}   # name -> (group key, column offset, C)
        self.shapes = {}   # group key -> (rows, width)
        self.bufs = {}
        self.init = {}

    def declare_group(self, key, rows, width, members):
        self.shapes[key] = (rows, width)
        self.members = getattr(self, "members", {})
        self.members[key] = list(members)
        for name, off, C in members:
            self.groups[name] = (key, off, C)

    def declare(self, name, rows, C):
        self.declare_group(name, rows, C, [(name, 0, C)])

    def get(self, name):
        key, off, C = self.groups[name]
        if key not in self.bufs:
            rows, width = self.shapes[key]
            self.bufs[key] = torch.empty(rows, width, dtype=torch.bfloat16, device=self.device)
        fresh = not self.init.get(name, False)
        self.init[name] = True
        for other, o2, c2 in getattr(self, "members", {}).get(key, ()):  # a written range initialises what it covers
            if off <= o2 and o2 + c2 <= off + C:
                self.init[other] = True
        return self.bufs[key][:, off:off + C], fresh

    def alias(self, name, view):
        """Let activation `name` use `view` (same shape, compact) as its gradient buffer."""
        self.bufs[name] = view
        self.groups[name] = (name, 0, view.shape[1])
        self.init[name] = True


class Tape(list):
    """Reverse-mode schedule; every entry is tagged with the block label it belongs to."""
    label = "input"

    def append(self, item):
        fn, c = item
        c["label"] = self.label
        super().append(item)


class UNetEngine:
    def __init__(self, cfg, params, grads=None, base=None, im_channels=4, single_stream=False):
        """params / grads: {state-dict key: fp32 CUDA tensor}; grads may be None (inference). single_stream: no side
        streams (weight gradients and the context branch inline)."""
        self.cfg = cfg
        self.L = layout(cfg)
        self.base = base or ("cond" if cfg.get("condition_config") else "uncond")
        self.P = _WaitingParams(params, self)
        self.Gd = grads
        # optimizer / pack pipeline: chunk -> event the current stream still has to wait for before it reads the
        # chunk's parameters or packed weights (set by the trainer after it issues the chunked optimizer step)
        self._pending = {}
        self._key_chunk = {}
        self.im_channels = im_channels
        self.device = next(iter(params.values())).device
        L = self.L
        # class conditioning (unet_cond_base.py:152-155): t_emb += class @ class_emb.weight, as one GEMM whose K
        # (the class count) is zero-padded to a multiple of 8
        self.kpad = (L["num_classes"] + 7) // 8 * 8 if L["klass"] else 0
        self.resnets = resnet_list(L)
        self.temb_off = {}
        off = 0
        for (p, l, cin, cout) in self.resnets:
            self.temb_off[(p, l)] = off
            off += cout
        self.temb_total = off
        # every cross-attention's context_proj (blocks.py context_proj: Linear(text_embed_dim, C)) reads the same
        # text context: their weights are one packed [sum C][ctx_dim] matrix (contiguous fp32 runs in the flat
        # store), so the forward is ONE GEMM into a [B*S][sum C] buffer and the weight gradient one GEMM at the end
        self.ctx_off, off = {}, 0
        for (p, l, c) in (cross_list(L) if L["text"] else []):
            self.ctx_off[(p, l)] = off
            off += c
        self.ctx_total = off
        # weight-gradient work (wgrad GEMMs, bias sums) runs on a side stream, overlapped with the
        # data-gradient chain of the backward on the current stream
        use_side = self.device.type == "cuda" and not single_stream
        self.side = streams.new_stream(self.device) if use_side else None
        # the weight-gradient blocks go round-robin over two side streams (the first is self.side, which also runs the
        # optimizer chunks), so independent small weight-gradient GEMMs overlap each other as well as the
        # data-gradient chain (measured 1 / 2 / 3 / 4 streams: 15.3-15.7 / 15.04-15.09 / 15.2 / 15.1-15.2 ms/step)
        self.sides = [self.side, streams.new_stream(self.device)] if use_side else []
        self._wg_next = 0
        # the cross-attention context branch runs ahead of the forward on a stream of its own
        self.ctx_stream = streams.new_stream(self.device) if use_side else None
        self._keep = []
        # linear data gradients from transposed packed weights: B_NK GEMMs, which the deep-ring 64-row mainloops of
        # the 8^2 / 4^2 levels take (round 2, before those mainloops: +0.04 ms/step; round 4 with the shapes tuned:
        # -0.14 ms/step, same-box A/B)
        self.dgrad_t = True
        self._build_pack()

    # ------------------------------------------------------------------------------------------
    def _build_pack(self):
        P, L = self.P, self.L
        pk = PackPlan(self.device)
        conv, lin = self._pk_conv, self._pk_lin

        cin_img = self.im_channels + (L["im_out"] if L["image"] else 0)
        self.cin_pad = (cin_img + 7) // 8 * 8
        first = "conv_in_concat" if L["image"] else "conv_in"
        self.first = first
        conv(pk, first, ipad=self.cin_pad)
        lin(pk, "t_proj.0")
        lin(pk, "t_proj.2")
        if L["klass"]:  # [classes (zero rows up to kpad)][T]: the B operand (k = class) of the class-embedding GEMM
            pk.add("class_emb#kn", P["class_emb.weight"], L["num_classes"], L["T"], L["T"], 1, 1, L["T"], 1, 0, 0,
                   rows=self.kpad)
        # concatenated t_emb_layers weight [sum C][T]
        pk.reserve("temb_all", self.temb_total, L["T"])
        for (p, l, cin, cout) in self.resnets:
            w = P[f"{p}.t_emb_layers.{l}.1.weight"]
            pk.add(None, w, cout, L["T"], L["T"], 1, 1, L["T"], 1, 0, 0, into="temb_all", row0=self.temb_off[(p, l)])
        if self.ctx_total:  # concatenated context_proj weight [sum C][ctx_dim]
            D = L["ctx_dim"]
            pk.reserve("ctxp_all", self.ctx_total, D)
            for (p, l, c) in self._cross_layers():
                w = P[f"{p}.context_proj.{l}.weight"]
                pk.add(None, w, c, D, D, 1, 1, D, 1, 0, 0, into="ctxp_all", row0=self.ctx_off[(p, l)])
        for (p, l, cin, cout) in self.resnets:
            self._pk_resnet(pk, p, l, cin, cout)
        nd = len(L["down"]) - 1
        for i in range(nd):
            p = f"downs.{i}"
            for l in range(L["n_down"]):
                if L["attn"][i]:
                    lin(pk, f"{p}.attentions.{l}.in_proj_weight")
                    lin(pk, f"{p}.attentions.{l}.out_proj")
                if L["text"]:
                    lin(pk, f"{p}.cross_attentions.{l}.in_proj_weight")
                    lin(pk, f"{p}.cross_attentions.{l}.out_proj")
            if L["down_sample"][i]:
                self._pk_down(pk, f"{p}.down_sample_conv")
        for i in range(len(L["mid"]) - 1):
            p = f"mids.{i}"
            for l in range(L["n_mid"]):
                lin(pk, f"{p}.attentions.{l}.in_proj_weight")
                lin(pk, f"{p}.attentions.{l}.out_proj")
                if L["text"]:
                    lin(pk, f"{p}.cross_attentions.{l}.in_proj_weight")
                    lin(pk, f"{p}.cross_attentions.{l}.out_proj")
        for j, i in enumerate(reversed(range(nd))):
            p = f"ups.{j}"
            for l in range(L["n_up"]):
                lin(pk, f"{p}.attentions.{l}.in_proj_weight")
                lin(pk, f"{p}.attentions.{l}.out_proj")
                if L["text"]:
                    lin(pk, f"{p}.cross_attentions.{l}.in_proj_weight")
                    lin(pk, f"{p}.cross_attentions.{l}.out_proj")
            if L["down_sample"][i]:
                self._pk_up(pk, f"{p}.up_sample_conv")
        conv(pk, "conv_out", opad=8)
        pk.finalize()
        self.pack = pk

    # ---- packed layouts (shared with the VQVAE training engine) --------------------------------------------
    def _pk_conv(self, pk, key, fwd=True, dgrad=True, ipad=None, opad=None):
        """key#f [O][KH][KW][Ipad] (forward) and key#d (stride-1 data gradient: flipped taps, transposed)."""
        w = self.P[key + ".weight"]
        O, I, KH, KW = w.shape
        Ip = ipad or I
        so, si, skh, skw = w.stride()  # torch (co, ci, kh, kw) or GEMM-natural (co, kh, kw, ci) memory order
        if fwd:
            pk.add(key + "#f", w, O, I, Ip, KH, KW, so, si, skh, skw, rows=opad)
        if dgrad and fwd:  # stride-1 dgrad [I][KH][KW][O] with flipped taps = the forward layout transposed
            pk.add_transpose(key + "#d", key + "#f", O, I, KH * KW, [KH * KW - 1 - t for t in range(KH * KW)], Ip,
                             rows=ipad, opad=opad)
        elif dgrad:
            pk.add(key + "#d", w, I, O, opad or O, KH, KW, si, so, skh, skw, KH - 1, -1, KW - 1, -1, rows=ipad)

    def _pk_lin(self, pk, key):
        w = self.P[key + ".weight"] if key + ".weight" in self.P else self.P[key]
        N, Kd = w.shape
        pk.add(key + "#f", w, N, Kd, Kd, 1, 1, Kd, 1, 0, 0)
        if self.dgrad_t:  # [Kd][N] for the data gradient (B_NK GEMM)
            pk.add_transpose(key + "#t", key + "#f", N, Kd, 1, [0], 8)

    def _pk_resnet(self, pk, p, l, cin, cout):
        P = self.P
        self._pk_conv(pk, f"{p}.resnet_conv_first.{l}.2")
        # second conv and the 1x1 residual conv as one K-concatenated weight [cout][9*cout + cin]
        w2 = P[f"{p}.resnet_conv_second.{l}.2.weight"]
        wr = P[f"{p}.residual_input_conv.{l}.weight"]
        cat = f"{p}.res{l}#cat"
        pk.reserve(cat, cout, 9 * cout + cin)
        pk.add(None, w2, cout, cout, cout, 3, 3, *w2.stride(), into=cat)
        pk.add(None, wr, cout, cin, cin, 1, 1, cin, 1, 0, 0, into=cat, col0=9 * cout)
        # its dgrad layout: the conv part of the concatenated forward weight, transposed per (flipped) tap
        pk.add_transpose(f"{p}.resnet_conv_second.{l}.2#d", cat, cout, cout, 9, [8 - t for t in range(9)], cout)
        if self.dgrad_t:  # the 1x1 residual conv's weight transposed [cin][cout] for its data gradient
            pk.add_transpose(f"{p}.res{l}#t", cat, cout, cin, 1, [0], 8, src_col0=9 * cout)

    def _pk_down(self, pk, key):
        """Stride-2 4x4 conv: key#f, plus its data gradient as four sub-pixel phases key#d{ph}{pw}."""
        C = self.P[key + ".weight"].shape[0]
        self._pk_conv(pk, key, dgrad=False)
        for ph in range(2):
            for pw in range(2):  # dgrad phases: [ci][a][b][co] = W[co][ci][3-ph-2a][3-pw-2b] = #f[co][tap][ci]
                pk.add_transpose(f"{key}#d{ph}{pw}", key + "#f", C, C, 4,
                                 [(3 - ph - 2 * a) * 4 + (3 - pw - 2 * b) for a in range(2) for b in range(2)], C)

    def _pk_up(self, pk, key):
        """ConvTranspose2d(4, 2, 1): key#d (its data gradient = a stride-2 conv over dY) and the forward as four
        sub-pixel phases key#f{ph}{pw}."""
        w = self.P[key + ".weight"]  # (Cx, Cy, 4, 4)
        Cx, Cy = w.shape[0], w.shape[1]
        # dgrad = stride-2 conv over dY: [ci][kh][kw][co] = W[ci][co][kh][kw]
        pk.add(f"{key}#d", w, Cx, Cy, Cy, 4, 4, Cy * 16, 16, 4, 1)
        for ph in range(2):
            for pw in range(2):  # fwd phases: [co][a][b][ci] = W[ci][co][3-ph-2a][3-pw-2b] = #d[ci][tap][co]
                pk.add_transpose(f"{key}#f{ph}{pw}", f"{key}#d", Cx, Cy, 4,
                                 [(3 - ph - 2 * a) * 4 + (3 - pw - 2 * b) for a in range(2) for b in range(2)], Cy)

    def W(self, name):
        if self._pending:
            self._need(self.pack.view_chunk.get(name, 0))
        return self.pack.view(name)

    def _dgrad(self, dy, key, out, **kw):
        """Data gradient of the packed linear `key` (#f [N][K]): from its transposed copy #t when packed."""
        if self.dgrad_t:
            K.linear_dgrad_t(dy, self.W(key + "#t"), out, **kw)
        else:
            K.linear_dgrad(dy, self.W(key + "#f"), out, **kw)

    def set_chunks(self, key_chunk):
        """Parameters are updated and repacked in forward-ordered chunks (trainer): key -> chunk index."""
        self._key_chunk = dict(key_chunk)
        ptr_chunk = {self.P.raw(k).data_ptr(): c for k, c in key_chunk.items()}
        self.pack.set_chunks(lambda ptr: ptr_chunk.get(ptr, 0), max(key_chunk.values()) + 1)

    def _need(self, c):
        ev = self._pending.pop(c, None)
        if ev is not None:
            plan.wait_event(torch.cuda.current_stream(self.device), ev)

    def _need_all(self):
        for c in sorted(self._pending):
            self._need(c)

    def refresh_weights(self):
        if self.pack.stale():
            self.pack.finalize()
        self.pack.run()

    # ------------------------------------------------------------------------------------------
    def _new(self, rows, C, dtype=torch.bfloat16):
        return torch.empty(rows, C, dtype=dtype, device=self.device)

    def g(self, key):
        return self.Gd[key] if self.Gd is not None else None

    def wperm(self, key):
        """conv_wgrad output layout of a conv weight gradient: torch (co, ci, kh, kw) order (column permute) for a
        contiguous gradient view, the GEMM's own (co, kh, kw, ci) order (16-B row stores) for a natural-order one
        (sdmi.store.unet_gemm_natural)."""
        return self.g(key).is_contiguous()

    def forward(self, x, t, text=None, mask=None, need_backward=True, mask_keep=None, klass=None, ctx_cache=None):
        """x: (B, C, H, W) fp32; t: int64 (B,), (1,) or 0-d; text: (B, S, ctx) ; mask: (B, cmi, MH, MW) fp32;
        klass: (B, num_classes) fp32 (one-hot, cond-drop already applied) for class-conditional configs;
        ctx_cache: context_cache() of the text (inference only: the context branch is then read, not recomputed).
        Returns (pred NHWC fp32 [B*H*W, 8] with the first im_channels valid, tape)."""
        L, P = self.L, self.P
        B, Cx, H, W = x.shape
        assert Cx == self.im_channels
        dev = self.device
        G, Hh = L["G"], L["heads"]
        K.PHASE = "fwd"
        tape = Tape()
        st = dict(B=B, H=H, W=W)
        grads = Grads(dev)
        self._grads = grads
        x = plan.as_operand(x)
        # ---- resolutions and concat buffers ----
        nd = len(L["down"]) - 1
        res = [(H, W)]
        for i in range(nd):
            h, w = res[-1]
            res.append((h // 2, w // 2) if L["down_sample"][i] else (h, w))
        cats = []
        for i in range(nd):
            h, w = res[i]
            C = L["down"][i]
            buf = self._new(B * h * w, 2 * C)
            cats.append(buf)
            grads.declare_group(f"cat{i}", B * h * w, 2 * C, [(f"up{i}", 0, C), (f"skip{i}", C, C), (f"cat{i}", 0, 2 * C)])

        # ---- input staging + first conv (unet_cond_base.py:131-140) ----
        xin = self._new(B * H * W, self.cin_pad)
        m = (plan.as_operand(mask, torch.uint8 if K.is_class_map(mask) else torch.float32) if L["image"] else None)
        K.prep_input(x, B, Cx, H, W, m, L.get("im_in", 0), P["cond_conv_in.weight"] if m is not None else None,
                     L.get("im_out", 0),
                     xin, self.cin_pad, mask_keep)
        skip0 = cats[0][:, L["down"][0]:]
        K.conv_fwd(xin, B, H, W, self.cin_pad, self.cin_pad, self.W(self.first + "#f"), L["down"][0], 3, 3, 1, 1,
                   skip0, K.ld_of(skip0), bias=P[self.first + ".bias"])
        tape.append((self._bwd_input, dict(xin=xin, mask=m, keep=mask_keep, B=B, H=H, W=W)))

        # ---- time embedding (blocks.py:5-24, unet_cond_base.py:148-149) ----
        tape.label = "time"
        T = L["T"]
        t = plan.timesteps(t, dev)
        if t.numel() not in (1, B):
            raise ValueError("t must have 1 or B elements")
        e = self._new(B, T)
        _lib.check(_lib.lib().sdmi_time_embedding(t.data_ptr(), 0 if t.numel() == 1 else 1, B, T, e.data_ptr(), T,
                                                  None, K._stream()), "sdmi_time_embedding")
        h1 = self._new(B, T)
        K.linear(e, self.W("t_proj.0#f"), h1, bias=P["t_proj.0.bias"])
        s1 = self._new(B, T)
        _lib.check(_lib.lib().sdmi_silu(h1.data_ptr(), None, s1.data_ptr(), B * T, K._stream()), "sdmi_silu")
        temb = self._new(B, T)
        K.linear(s1, self.W("t_proj.2#f"), temb, bias=P["t_proj.2.bias"])
        cls = None
        if L["klass"]:
            if klass is None:
                raise ValueError("class-conditional model: klass (B, num_classes) is required")
            kl = plan.as_operand(klass)
            if tuple(kl.shape) != (B, L["num_classes"]):
                raise ValueError(f"klass must be (B, {L['num_classes']})")
            cls = self._new(B, self.kpad)
            _lib.check(_lib.lib().sdmi_nchw_to_nhwc_bf16(kl.data_ptr(), B, L["num_classes"], 1, cls.data_ptr(),
                                                         self.kpad, K._stream()), "cast")
            # temb += class @ class_emb.weight (in-place residual epilogue)
            K.gemm(B, T, self.kpad, cls, _lib.A_ROWMAJOR, self.kpad, self.W("class_emb#kn"), _lib.B_KN, T, temb, T,
                   resid=temb, ldr=T)
        stemb = self._new(B, T)
        _lib.check(_lib.lib().sdmi_silu(temb.data_ptr(), None, stemb.data_ptr(), B * T, K._stream()), "sdmi_silu")
        temb_all = self._new(B, self.temb_total)
        # biases of all t_emb_layers: gathered once per call into a contiguous fp32 vector
        bias_all = self._temb_bias()
        K.linear(stemb, self.W("temb_all"), temb_all, bias=bias_all)
        self.dtemb_all = None
        time_c = dict(e=e, h1=h1, s1=s1, temb=temb, stemb=stemb, B=B, cls=cls)
        tape.append((self._bwd_time, time_c))
        st["temb_all"] = temb_all

        ctx = None
        if L["text"] and ctx_cache is not None:
            if need_backward:
                raise ValueError("ctx_cache is an inference-only input (the backward needs the step's own context)")
            if ctx_cache["B"] != B:
                raise ValueError(f"ctx_cache was built for B={ctx_cache['B']}, forward has B={B}")
            ctx = ctx_cache["ctx"]
            st.update(S=ctx_cache["S"], cp_all=ctx_cache["cp_all"], kv_cache=ctx_cache["kv"])
        elif L["text"]:
            txt = plan.as_operand(text)
            S = txt.shape[1]
            ctx = self._new(B * S, txt.shape[2])
            _lib.check(_lib.lib().sdmi_nchw_to_nhwc_bf16(txt.data_ptr(), B * S, txt.shape[2], 1, ctx.data_ptr(),
                                                         txt.shape[2], K._stream()), "cast")
            st["S"] = S
        st["ctx"] = ctx
        time_c["ctx"] = ctx
        # inference (no backward) keeps the context branch inline: the sampler's reverse step measured 1.75 vs 2.02 ms
        # at B = 1 and 2.51 vs 2.64 ms at B = 8 (scripts/sample_graph_probe.py) -- its small launches gain nothing
        # from running beside the forward and the stream's event edges cost a dispatch each; it also keeps the step
        # one stream, which a hipGraph replays as one batch (multi-stream graphs replay at eager host cost)
        if ctx_cache is not None:
            pass
        elif ctx is not None and self.ctx_stream is not None and need_backward:
            self._ctx_ahead(st, B)
        elif ctx is not None:  # every context_proj in one GEMM (inline context branch)
            st["cp_all"] = self._new(B * st["S"], self.ctx_total)
            K.linear(ctx, self.W("ctxp_all"), st["cp_all"], bias=self._ctx_bias(self.P))

        # ---- down blocks (blocks.py:111-146) ----
        cur, cur_name = skip0, "skip0"
        for i in range(nd):
            p = f"downs.{i}"
            tape.label = p
            h, w = res[i]
            cin, cout = L["down"][i], L["down"][i + 1]
            ops = []
            for l in range(L["n_down"]):
                ops.append(("res", l, cin if l == 0 else cout))
                if L["attn"][i]:
                    ops.append(("self", l, cout))
                if L["text"]:
                    ops.append(("cross", l, cout))
            if L["down_sample"][i]:
                ops.append(("down", 0, cout))
            # where the block's output goes: the next concat's skip half, or a fresh buffer for the mids
            dst_name = f"skip{i + 1}" if i + 1 < nd else "mid_in"
            for k, (kind, l, c) in enumerate(ops):
                last = k == len(ops) - 1
                out = None
                oname = f"{p}.{kind}{l}"
                if last:
                    if i + 1 < nd:
                        out = cats[i + 1][:, L["down"][i + 1]:]
                    oname = dst_name
                cur, cur_name = self._op(kind, p, l, c, cout, cur, cur_name, out, oname, B, h, w, st, tape, grads)

        # ---- mid blocks (blocks.py:225-267) ----
        h, w = res[-1]
        for i in range(len(L["mid"]) - 1):
            p = f"mids.{i}"
            tape.label = p
            cin, cout = L["mid"][i], L["mid"][i + 1]
            cur, cur_name = self._op("res", p, 0, cin, cout, cur, cur_name, None, f"{p}.res0", B, h, w, st, tape, grads)
            for l in range(L["n_mid"]):
                cur, cur_name = self._op("self", p, l, cout, cout, cur, cur_name, None, f"{p}.self{l}", B, h, w, st,
                                         tape, grads)
                if L["text"]:
                    cur, cur_name = self._op("cross", p, l, cout, cout, cur, cur_name, None, f"{p}.cross{l}", B, h, w,
                                             st, tape, grads)
                cur, cur_name = self._op("res", p, l + 1, cout, cout, cur, cur_name, None, f"{p}.res{l + 1}", B, h,
                                         w, st, tape, grads)

        # ---- up blocks (blocks.py:461-499) ----
        for j, i in enumerate(reversed(range(nd))):
            p = f"ups.{j}"
            tape.label = p
            h, w = res[i]
            C = L["down"][i]
            up_view = cats[i][:, :C]
            if L["down_sample"][i]:
                self._op("up", p, 0, C, C, cur, cur_name, up_view, f"up{i}", B, res[i + 1][0], res[i + 1][1], st,
                         tape, grads)
            else:
                K.copy_slice(cur, up_view)
                tape.append((self._bwd_copy, dict(src=cur_name, dst=f"up{i}")))
            cur, cur_name = cats[i], f"cat{i}"
            cin = 2 * C
            cout = L["down"][i - 1] if i != 0 else L["conv_out"]
            for l in range(L["n_up"]):
                cur, cur_name = self._op("res", p, l, cin if l == 0 else cout, cout, cur, cur_name, None, f"{p}.res{l}",
                                         B, h, w, st, tape, grads)
                cur, cur_name = self._op("self", p, l, cout, cout, cur, cur_name, None, f"{p}.self{l}", B, h, w, st,
                                         tape, grads)
                if L["text"]:
                    cur, cur_name = self._op("cross", p, l, cout, cout, cur, cur_name, None, f"{p}.cross{l}", B, h, w,
                                             st, tape, grads)

        # ---- head (unet_cond_base.py:179-181) ----
        tape.label = "head"
        C = L["conv_out"]
        Pn = H * W
        hs = self._new(B * Pn, C)
        tab = K.gn_fwd(cur, B, Pn, C, G, P["norm_out.weight"], P["norm_out.bias"], True, hs)
        pred = self._new(B * Pn, 8, torch.float32)
        K.conv_fwd(hs, B, H, W, C, C, self.W("conv_out#f"), 8, 3, 3, 1, 1, pred, 8, bias=P["conv_out.bias"],
                   n_store=self.im_channels)
        tape.append((self._bwd_head, dict(x=cur, xn=cur_name, tab=tab, hs=hs, B=B, H=H, W=W)))
        return pred, dict(tape=tape, st=st, grads=grads) if need_backward else None

    # ------------------------------------------------------------------------------------------
    def _cross_layers(self):
        """(block prefix, layer, channels) of every cross-attention, in forward order."""
        return cross_list(self.L)

    def _wait_chunk_on(self, stream, c):
        ev = self._pending.get(c)  # (not popped: the current stream still waits for it where it reads the chunk)
        if ev is not None:
            plan.wait_event(stream, ev)

    def _ctx_ahead(self, st, B):
        """The context branch of every cross-attention -- context_proj (all layers in ONE GEMM of the text context
        against the concatenated [sum C][ctx_dim] weight), then the k|v rows of each attention's packed
        in-projection (blocks.py:139-140 -> nn.MultiheadAttention) -- depends only on the text context: issue all of
        it up front on a stream of its own, each GEMM waiting for the optimizer chunks that update its weights, so
        its launches run beside the forward's main chain instead of on it. The buffers are allocated on the current
        stream (which waits for each layer's event before its attention reads them)."""
        P, S, ctx = self.P, st["S"], st["ctx"]
        cs = self.ctx_stream
        cp_all = self._new(B * S, self.ctx_total)
        work = []
        for (p, l, C) in self._cross_layers():
            work.append((p, l, C, self._new(B * S, 2 * C)))
        plan.wait_stream(cs, torch.cuda.current_stream(self.device))
        pre = {}
        with torch.cuda.stream(cs):
            self._wait_chunk_on(cs, self.pack.view_chunk.get("ctxp_all", 0))
            for c in sorted({self._key_chunk.get(k, 0) for k in self._ctx_bias_keys()}):
                self._wait_chunk_on(cs, c)
            # raw parameter reads: the waits above are on the context stream; the main stream keeps its own
            raw = {k: P.raw(k) for k in self._ctx_bias_keys()}
            K.linear(ctx, self.pack.view("ctxp_all"), cp_all, bias=self._ctx_bias(raw))
            for (p, l, C, kv) in work:
                mk = f"{p}.cross_attentions.{l}"
                self._wait_chunk_on(cs, self.pack.view_chunk.get(mk + ".in_proj_weight#f", 0))
                self._wait_chunk_on(cs, self._key_chunk.get(mk + ".in_proj_bias", 0))
                off = self.ctx_off[(p, l)]
                cp = cp_all[:, off:off + C]
                K.linear(cp, self.pack.view(mk + ".in_proj_weight#f")[C:], kv, bias=P.raw(mk + ".in_proj_bias")[C:])
                ev = torch.cuda.Event()
                plan.record_event(ev, cs)
                pre[(p, l)] = (cp, kv, ev)
        st["cp_all"] = cp_all
        st["ctx_pre"] = pre

    def context_cache(self, text, cache=None):
        """The forward's context branch -- the text context cast to bf16, every context_proj (ONE GEMM) and every
        cross-attention's k|v rows of its packed in-projection (blocks.py:139-140) -- depends only on the text and
        the weights. A sampling loop (one condition for all its steps) computes it once per run with this and passes
        it to forward(ctx_cache=...); `cache` (a previous result) is refilled in place, so a captured step keeps
        reading the same memory. The launches are the inline branch's own (same shapes, phase and tiles), so the
        forward's output is bitwise the uncached one's. Returns the cache, or None for a model without text."""
        if not self.L["text"]:
            return None
        B, S, D = text.shape
        if cache is None:
            cache = dict(B=B, S=S, ctx=self._new(B * S, D), cp_all=self._new(B * S, self.ctx_total),
                         kv={(p, l): self._new(B * S, 2 * C) for (p, l, C) in self._cross_layers()})
        elif (cache["B"], cache["S"], cache["ctx"].shape[1]) != (B, S, D):
            raise ValueError("context_cache: text shape differs from the cached one")
        txt = text.float().contiguous()
        K.PHASE = "fwd"
        _lib.check(_lib.lib().sdmi_nchw_to_nhwc_bf16(txt.data_ptr(), B * S, D, 1, cache["ctx"].data_ptr(), D,
                                                     K._stream()), "cast")
        K.linear(cache["ctx"], self.W("ctxp_all"), cache["cp_all"], bias=self._ctx_bias(self.P))
        for (p, l, C) in self._cross_layers():
            mk = f"{p}.cross_attentions.{l}"
            off = self.ctx_off[(p, l)]
            K.linear(cache["cp_all"][:, off:off + C], self.W(mk + ".in_proj_weight#f")[C:], cache["kv"][(p, l)],
                     bias=self.P[mk + ".in_proj_bias"][C:])
        return cache

    def _ctx_bias_keys(self):
        return [f"{p}.context_proj.{l}.bias" for (p, l, c) in self._cross_layers()]

    def _ctx_bias(self, params):
        """The context_proj biases are one contiguous fp32 vector of the flat store (layer order)."""
        return contiguous_run(params, self._ctx_bias_keys(), (self.ctx_total,))

    def _temb_bias(self):
        """The t_emb_layers biases are one contiguous fp32 vector of the flat store (forward order)."""
        return contiguous_run(self.P, [f"{p}.t_emb_layers.{l}.1.bias" for (p, l, ci, co) in self.resnets],
                              (self.temb_total,))

    def _op(self, kind, p, l, cin, cout, x, xname, out, oname, B, h, w, st, tape, grads):
        if kind == "res":
            y = self._resnet_fwd(p, l, cin, cout, x, xname, out, oname, B, h, w, st, tape)
        elif kind == "self":
            y = self._attn_fwd(p, l, cout, x, xname, out, oname, B, h, w, st, tape, cross=False)
        elif kind == "cross":
            y = self._attn_fwd(p, l, cout, x, xname, out, oname, B, h, w, st, tape, cross=True)
        elif kind == "down":
            y = self._down_fwd(p, cout, x, xname, out, oname, B, h, w, tape)
        elif kind == "up":
            y = self._up_fwd(p, cin, x, xname, out, oname, B, h, w, tape)
        else:
            raise ValueError(kind)
        if oname not in grads.groups:
            grads.declare(oname, y.shape[0], y.shape[1])
        return y, oname

    # ---- resnet ----------------------------------------------------------------------------------
    def _resnet_fwd(self, p, l, cin, cout, x, xname, out, oname, B, h, w, st, tape):
        P, G = self.P, self.L["G"]
        Pn = h * w
        a, b = f"{p}.resnet_conv_first.{l}", f"{p}.resnet_conv_second.{l}"
        h0 = self._new(B * Pn, cin)
        t1 = K.gn_fwd(x, B, Pn, cin, G, P[a + ".0.weight"], P[a + ".0.bias"], True, h0)
        h1 = self._new(B * Pn, cout)
        off = self.temb_off.get((p, l))  # None: no time embedding (the VQVAE's blocks, t_emb_dim=None)
        K.conv_fwd(h0, B, h, w, cin, cin, self.W(a + ".2#f"), cout, 3, 3, 1, 1, h1, cout, bias=P[a + ".2.bias"],
                   rowbias=st["temb_all"][:, off:] if off is not None else None, rb_ld=self.temb_total)
        h2 = self._new(B * Pn, cout)
        t2 = K.gn_fwd(h1, B, Pn, cout, G, P[b + ".0.weight"], P[b + ".0.bias"], True, h2)
        rc = f"{p}.residual_input_conv.{l}"
        y = out if out is not None else self._new(B * Pn, cout)
        # conv2(h2) + residual 1x1(x) in ONE GEMM: A = [im2col(h2) | x], B = [W2 | Wr]
        K.conv_fwd(h2, B, h, w, cout, cout, self.W(f"{p}.res{l}#cat"), cout, 3, 3, 1, 1, y, K.ld_of(y),
                   bias=P[b + ".2.bias"], x2=x, cin2=cin, bias2=P[rc + ".bias"])
        tape.append((self._resnet_bwd, dict(p=p, l=l, cin=cin, cout=cout, x=x, xn=xname, yn=oname, h0=h0, h1=h1, h2=h2,
                                            t1=t1, t2=t2, B=B, h=h, w=w)))
        return y

    def _resnet_bwd(self, c, grads):
        P, G = self.P, self.L["G"]
        p, l, cin, cout, B, h, w = c["p"], c["l"], c["cin"], c["cout"], c["B"], c["h"], c["w"]
        Pn = h * w
        a, b = f"{p}.resnet_conv_first.{l}", f"{p}.resnet_conv_second.{l}"
        rc = f"{p}.residual_input_conv.{l}"
        dy, _ = grads.get(c["yn"])
        ldy = K.ld_of(dy)
        with self._wg(dy):
            # conv2 and residual-conv bias gradients (both = column sums of dy) come out of the same launch
            K.conv_wgrad(dy, ldy, c["h2"], B, h, w, cout, cout, cout, 3, 3, 1, 1, self.g(b + ".2.weight"), h, w,
                         perm=self.wperm(b + ".2.weight"), bias_grad=self.g(b + ".2.bias"),
                         bias_grad2=self.g(rc + ".bias"))
        self._wgrad_linear(dy, c["x"], self.g(rc + ".weight").view(cout, cin))
        dh2 = self._new(B * Pn, cout)
        # the GroupNorm backward's reductions come out of the data-gradient GEMM that produces its input gradient
        g2 = _gn_req(c["h1"], c["t2"], Pn, cout, True)
        K.conv_fwd(dy, B, h, w, cout, ldy, self.W(b + ".2#d"), cout, 3, 3, 1, 1, dh2, cout, gn=g2)
        dx, fresh = grads.get(c["xn"])
        if self.dgrad_t:
            K.linear_dgrad_t(dy, self.W(f"{p}.res{l}#t"), dx, resid=None if fresh else dx)
        else:
            K.linear_dgrad(dy, self.W(f"{p}.res{l}#cat")[:, 9 * cout:], dx, resid=None if fresh else dx)
        K.gn_bwd(c["h1"], dh2, dh2, c["t2"], P[b + ".0.weight"], B, Pn, cout, G, True,
                 self.g(b + ".0.weight"), self.g(b + ".0.bias"), gn=g2, defer=self._gn_defer())
        off = self.temb_off.get((p, l))
        with self._wg(dh2):
            # conv1 bias, t_emb_layers bias and the per-sample time-embedding gradient (blocks.py:117-118) are
            # reductions of dh2 computed by the weight-gradient launch itself
            K.conv_wgrad(dh2, cout, c["h0"], B, h, w, cin, cin, cout, 3, 3, 1, 1, self.g(a + ".2.weight"), h, w,
                         perm=self.wperm(a + ".2.weight"), bias_grad=self.g(a + ".2.bias"),
                         bias_grad2=self.g(f"{p}.t_emb_layers.{l}.1.bias") if off is not None else None,
                         group_sums=self.dtemb_all[:, off:off + cout] if off is not None else None)
        if off is not None:
            self._note_time_input()
        dh0 = self._new(B * Pn, cin)
        g1 = _gn_req(c["x"], c["t1"], Pn, cin, True)
        K.conv_fwd(dh2, B, h, w, cout, cout, self.W(a + ".2#d"), cin, 3, 3, 1, 1, dh0, cin, gn=g1)
        K.gn_bwd(c["x"], dh0, dx, c["t1"], P[a + ".0.weight"], B, Pn, cin, G, True,
                 self.g(a + ".0.weight"), self.g(a + ".0.bias"), addend=dx, gn=g1, defer=self._gn_defer())

    # ---- self / cross attention --------------------------------------------------------------------
    def _attn_fwd(self, p, l, C, x, xname, out, oname, B, h, w, st, tape, cross):
        P, G, Hh = self.P, self.L["G"], self.L["heads"]
        N = h * w
        nk = f"{p}.cross_attention_norms.{l}" if cross else f"{p}.attention_norms.{l}"
        mk = f"{p}.cross_attentions.{l}" if cross else f"{p}.attentions.{l}"
        a = self._new(B * N, C)
        tab = K.gn_fwd(x, B, N, C, G, P[nk + ".weight"], P[nk + ".bias"], False, a)
        Win = self.W(mk + ".in_proj_weight#f")
        bin_ = P[mk + ".in_proj_bias"]
        d = C // Hh
        o = self._new(B * N, C)
        c = dict(p=p, l=l, C=C, x=x, xn=xname, yn=oname, a=a, tab=tab, o=o, B=B, N=N, cross=cross, nk=nk, mk=mk)
        if not cross:
            qkv = self._new(B * N, 3 * C)
            K.linear(a, Win, qkv, bias=bin_)
            c["lse"] = K.attn_fwd(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], o, B, Hh, N, N, d)
            c["qkv"] = qkv
        else:
            S = st["S"]
            ctx = st["ctx"]
            ck = f"{p}.context_proj.{l}"
            q = self._new(B * N, C)
            K.linear(a, Win[:C], q, bias=bin_[:C])
            pre = st.get("ctx_pre")
            if pre is not None:  # issued ahead on the context stream (_ctx_ahead)
                cp, kv, ev = pre[(p, l)]
                plan.wait_event(torch.cuda.current_stream(self.device), ev)
            elif st.get("kv_cache") is not None:  # computed once per sampling run (context_cache)
                off = self.ctx_off[(p, l)]
                cp = st["cp_all"][:, off:off + C]
                kv = st["kv_cache"][(p, l)]
            else:
                off = self.ctx_off[(p, l)]
                cp = st["cp_all"][:, off:off + C]
                kv = self._new(B * S, 2 * C)
                K.linear(cp, Win[C:], kv, bias=bin_[C:])
            c["lse"] = K.attn_fwd(q, kv[:, :C], kv[:, C:], o, B, Hh, N, S, d)
            c.update(q=q, cp=cp, kv=kv, S=S, ctx=ctx, ck=ck)
        y = out if out is not None else self._new(B * N, C)
        K.linear(o, self.W(mk + ".out_proj#f"), y, bias=P[mk + ".out_proj.bias"], resid=x)
        tape.append((self._attn_bwd, c))
        return y

    def _attn_bwd(self, c, grads):
        P, G, Hh = self.P, self.L["G"], self.L["heads"]
        C, B, N, mk, nk = c["C"], c["B"], c["N"], c["mk"], c["nk"]
        d = C // Hh
        dy, _ = grads.get(c["yn"])
        self._wgrad_linear(dy, c["o"], self.g(mk + ".out_proj.weight"), self.g(mk + ".out_proj.bias"))
        dy_read = self.wg_event if (self.side is not None and not self._grouping()) else None
        do = self._new(B * N, C)
        self._dgrad(dy, mk + ".out_proj", do)
        Win = self.W(mk + ".in_proj_weight#f")
        WinT = self.W(mk + ".in_proj_weight#t") if self.dgrad_t else None
        gW = self.g(mk + ".in_proj_weight")
        gb = self.g(mk + ".in_proj_bias")
        da = self._new(B * N, C)
        ga = _gn_req(c["x"], c["tab"], N, C, False)
        if not c["cross"]:
            qkv = c["qkv"]
            dqkv = self._new(B * N, 3 * C)
            K.attn_bwd(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], c["o"], do, c["lse"], dqkv[:, :C],
                       dqkv[:, C:2 * C], dqkv[:, 2 * C:], B, Hh, N, N, d)
            self._wgrad_linear(dqkv, c["a"], gW, gb)
            if WinT is not None:
                K.linear_dgrad_t(dqkv, WinT, da, gn=ga)
            else:
                K.linear_dgrad(dqkv, Win, da, gn=ga)
        else:
            S, kv = c["S"], c["kv"]
            dq = self._new(B * N, C)
            dkv = self._new(B * S, 2 * C)
            K.attn_bwd(c["q"], kv[:, :C], kv[:, C:], c["o"], do, c["lse"], dq, dkv[:, :C], dkv[:, C:], B, Hh, N, S, d)
            # the context branch (kv in-projection -> context_proj) ends at the text input, which takes no gradient:
            # its data gradient only feeds the context_proj weight gradient, so all of it runs on the side stream
            # this layer's columns of the shared context_proj output gradient (one weight-gradient GEMM for every
            # layer at the end of the backward, _bwd_time)
            off = self.ctx_off[(c["p"], c["l"])]
            dcp = self.dcp_all[:, off:off + C]
            self._wgrad_linear(dq, c["a"], gW[:C], gb[:C])
            self._wgrad_linear(dkv, c["cp"], gW[C:], gb[C:])
            with self._wg(dkv):
                if WinT is not None:
                    K.linear_dgrad_t(dkv, WinT[:, C:], dcp)
                else:
                    K.linear_dgrad(dkv, Win[C:], dcp)
            self._note_time_input()
            if WinT is not None:
                K.linear_dgrad_t(dq, WinT[:, :C], da, gn=ga)
            else:
                K.linear_dgrad(dq, Win[:C], da, gn=ga)
        # x receives dy (residual) + GroupNorm-branch gradient
        key, off, _ = grads.groups[c["xn"]]
        # (no alias while weight gradients are grouped: the deferred out_proj gradient still has to read dy)
        if self._dy_alias and not self._grouping() and not grads.init.get(c["xn"], False) and dy.is_contiguous() and \
                K.ld_of(dy) == C and grads.shapes.get(key, (0, 0))[1] == C:
            grads.alias(c["xn"], dy)
            dx, addend = dy, dy
            if dy_read is not None:  # the GroupNorm backward below rewrites dy in place
                plan.wait_event(torch.cuda.current_stream(self.device), dy_read)
        else:
            dx, fresh = grads.get(c["xn"])
            if not fresh:
                K.copy_slice(dy, dx, accumulate=True)
                addend = dx
            else:
                addend = dy
        K.gn_bwd(c["x"], da, dx, c["tab"], P[nk + ".weight"], B, N, C, G, False,
                 self.g(nk + ".weight"), self.g(nk + ".bias"), addend=addend, gn=ga, defer=self._gn_defer())

    # ---- down / up sampling convs --------------------------------------------------------------------
    def _down_fwd(self, p, C, x, xname, out, oname, B, h, w, tape):
        key = f"{p}.down_sample_conv"
        y = out if out is not None else self._new(B * (h // 2) * (w // 2), C)
        K.conv_fwd(x, B, h, w, C, K.ld_of(x), self.W(key + "#f"), C, 4, 4, 2, 1, y, K.ld_of(y),
                   bias=self.P[key + ".bias"])
        tape.append((self._down_bwd, dict(key=key, C=C, x=x, xn=xname, yn=oname, B=B, h=h, w=w)))
        return y

    def _down_bwd(self, c, grads):
        key, C, B, h, w = c["key"], c["C"], c["B"], c["h"], c["w"]
        dy, _ = grads.get(c["yn"])
        ldy = K.ld_of(dy)
        with self._wg(dy):
            K.conv_wgrad(dy, ldy, c["x"], B, h, w, C, K.ld_of(c["x"]), C, 4, 4, 2, 1, self.g(key + ".weight"),
                         h // 2, w // 2, perm=self.wperm(key + ".weight"), bias_grad=self.g(key + ".bias"))
        dx, fresh = grads.get(c["xn"])
        wph = [self.W(f"{key}#d{ph}{pw}") for ph in range(2) for pw in range(2)]
        K.conv_dgrad_phases(dy, B, h, w, C, ldy, wph, C, dx, K.ld_of(dx), resid=None if fresh else dx,
                            ldr=K.ld_of(dx))

    def _up_fwd(self, p, C, x, xname, out, oname, B, h, w, tape):
        key = f"{p}.up_sample_conv"
        wph = [self.W(f"{key}#f{ph}{pw}") for ph in range(2) for pw in range(2)]
        K.convT_fwd_phases(x, B, h, w, C, K.ld_of(x), wph, C, out, K.ld_of(out), bias=self.P[key + ".bias"])
        tape.append((self._up_bwd, dict(key=key, C=C, x=x, xn=xname, yn=oname, B=B, h=h, w=w)))
        return out

    def _up_bwd(self, c, grads):
        key, C, B, h, w = c["key"], c["C"], c["B"], c["h"], c["w"]
        dy, _ = grads.get(c["yn"])  # (B, 2h, 2w, C) slice of the concat gradient
        ldy = K.ld_of(dy)
        x = c["x"]
        with self._wg(dy):
            K.chan_sum(dy, B, 4 * h * w, C, per_c=self.g(key + ".bias"))
            # dW[ci][co][kh][kw] = sum_{pixels of x} x[p][ci] * dy[2*iy-1+kh, 2*ix-1+kw][co]
            g = K.conv_geom(2 * h, 2 * w, C, ldy, 4, 4, h, w, 2, 2, -1, -1)
            K.gemm(C, 16 * C, B * h * w, x, _lib.A_COLMAJOR, K.ld_of(x), dy, _lib.B_KN_CONV, 0,
                   self.g(key + ".weight"), 16 * C, geom=g, perm=(C, 16))
        dx, fresh = grads.get(c["xn"])
        K.conv_fwd(dy, B, 2 * h, 2 * w, C, ldy, self.W(key + "#d"), C, 4, 4, 2, 1, dx, K.ld_of(dx),
                   resid=None if fresh else dx, ldr=K.ld_of(dx))

    def _bwd_copy(self, c, grads):
        dy, _ = grads.get(c["dst"])
        dx, fresh = grads.get(c["src"])
        K.copy_slice(dy, dx, accumulate=not fresh)

    # ---- head / input / time embedding backward ------------------------------------------------------
    def _bwd_head(self, c, grads):
        P, G = self.P, self.L["G"]
        B, H, W = c["B"], c["H"], c["W"]
        C = self.L["conv_out"]
        Pn = H * W
        dpred = self.dpred
        with self._wg(dpred):
            K.conv_wgrad(dpred, 8, c["hs"], B, H, W, C, C, 8, 3, 3, 1, 1, self.g("conv_out.weight"), H, W,
                         m_store=self.im_channels, bias_grad=self.g("conv_out.bias"))
        dhs = self._new(B * Pn, C)
        gh = _gn_req(c["x"], c["tab"], Pn, C, True)
        K.conv_fwd(dpred, B, H, W, 8, 8, self.W("conv_out#d"), C, 3, 3, 1, 1, dhs, C, gn=gh)
        dx, fresh = grads.get(c["xn"])
        K.gn_bwd(c["x"], dhs, dx, c["tab"], P["norm_out.weight"], B, Pn, C, G, True,
                 self.g("norm_out.weight"), self.g("norm_out.bias"), addend=None if fresh else dx, gn=gh,
                 defer=self._gn_defer())

    def _bwd_input(self, c, grads):
        L = self.L
        B, H, W = c["B"], c["H"], c["W"]
        dy, _ = grads.get("skip0")
        ldy = K.ld_of(dy)
        C0 = L["down"][0]
        cin_real = self.im_channels + (L["im_out"] if L["image"] else 0)
        with self._wg(dy):
            K.conv_wgrad(dy, ldy, c["xin"], B, H, W, self.cin_pad, self.cin_pad, C0, 3, 3, 1, 1,
                         self.g(self.first + ".weight"), H, W, cvalid=cin_real, bias_grad=self.g(self.first + ".bias"))
        if L["image"]:
            dxin = self._new(B * H * W, self.cin_pad)
            K.conv_fwd(dy, B, H, W, C0, ldy, self.W(self.first + "#d"), self.cin_pad, 3, 3, 1, 1, dxin, self.cin_pad)
            K.cond_wgrad(dxin, self.cin_pad, self.im_channels, B, H, W, c["mask"], L["im_in"], L["im_out"],
                         self.g("cond_conv_in.weight"), c["keep"])

    def _bwd_time(self, c, grads):
        P, L = self.P, self.L
        B, T = c["B"], L["T"]
        # dtemb_all is filled by the resnets' side-stream weight-gradient launches and dcp_all by the cross-attentions'
        # side-stream data gradients: wait for exactly those, so the time-MLP backward overlaps the rest of the
        # weight-gradient backlog (backward() joins every side stream at its end). Same box, against joining every
        # side stream here: 13.41 / 13.44 and 13.42 / 13.34 vs 13.69 / 13.64 and 13.63 / 13.61 ms per step
        for ev in self._time_inputs:
            plan.wait_event(torch.cuda.current_stream(self.device), ev)
        self._time_inputs = []
        if c.get("ctx") is not None:  # every context_proj weight / bias gradient in one GEMM (contiguous runs)
            with self._wg(self.dcp_all):
                K.linear_wgrad(self.dcp_all, c["ctx"], self._ctx_grad_view(),
                               bias_grad=self._ctx_bias(self.Gd))
        d_all = self.dtemb_all
        # t_emb_layers weights are contiguous in the gradient store: one GEMM for all of them
        K.linear_wgrad(d_all, c["stemb"], self.temb_grad_all)
        dst = self._new(B, T)
        K.linear_dgrad(d_all, self.W("temb_all"), dst)
        dtemb = self._new(B, T)
        lib = _lib.lib()
        _lib.check(lib.sdmi_silu(c["temb"].data_ptr(), dst.data_ptr(), dtemb.data_ptr(), B * T, K._stream()), "silu")
        if c.get("cls") is not None:  # d class_emb.weight = class^T @ dtemb (A = the bf16 class rows, col-major)
            K.gemm(self.kpad, T, B, c["cls"], _lib.A_COLMAJOR, self.kpad, dtemb, _lib.B_KN, T,
                   self.g("class_emb.weight"), T, m_store=L["num_classes"])
        K.linear_wgrad(dtemb, c["s1"], self.g("t_proj.2.weight"), bias_grad=self.g("t_proj.2.bias"))
        ds1 = self._new(B, T)
        K.linear_dgrad(dtemb, self.W("t_proj.2#f"), ds1)
        dh1 = self._new(B, T)
        _lib.check(lib.sdmi_silu(c["h1"].data_ptr(), ds1.data_ptr(), dh1.data_ptr(), B * T, K._stream()), "silu")
        K.linear_wgrad(dh1, c["e"], self.g("t_proj.0.weight"), bias_grad=self.g("t_proj.0.bias"))

    # ------------------------------------------------------------------------------------------
    def loss(self, pred, noise, dpred, loss_out, gscale_dev=None, gscale=1.0):
        """nn.MSELoss(pred, noise) with pred NHWC fp32 [B*H*W, 8]; dpred (bf16, same layout) = dL/dpred."""
        B, C, H, W = noise.shape
        K.mse(pred, 8, noise, B, C, H * W, gscale, dpred, loss_out, gscale_dev=gscale_dev)

    def pred_to_nchw(self, pred, B, H, W):
        out = torch.empty(B, self.im_channels, H, W, dtype=torch.float32, device=self.device)
        _lib.check(_lib.lib().sdmi_nhwc_to_nchw(pred.data_ptr(), 1, 8, B, self.im_channels, H * W, out.data_ptr(),
                                                K._stream()), "sdmi_nhwc_to_nchw")
        return out

    def dpred_from_nchw(self, d):
        B, C, H, W = d.shape
        dpred = torch.empty(B * H * W, 8, dtype=torch.bfloat16, device=self.device)
        _lib.check(_lib.lib().sdmi_nchw_to_nhwc_bf16(d.data_ptr(), B, C, H * W, dpred.data_ptr(), 8, K._stream()),
                   "sdmi_nchw_to_nhwc_bf16")
        return dpred

    def new_dpred(self, B, H, W):
        return torch.empty(B * H * W, 8, dtype=torch.bfloat16, device=self.device)

    # ------------------------------------------------------------------------------------------
    @contextlib.contextmanager
    def _wg(self, *keep, balance=False):
        """Weight-gradient work: issued on the side stream after everything issued so far on the current
        stream. `keep` pins the operand tensors until the backward's final join, so the caching
        allocator cannot hand their memory to the current stream while the side stream still reads it.
        The block's completion event is left in self.wg_event. balance: the side stream with the fewer GEMM FLOPs
        issued so far in this backward (the block flushes' grouped launches), else round-robin."""
        prev = K.PHASE
        K.PHASE = "wg"
        if self.side is None:
            try:
                yield
            finally:
                K.PHASE = prev
            return
        self._keep.extend(keep)
        sflops = self.__dict__.setdefault("_side_flops", [0.0] * len(self.sides))  # reset per backward
        if balance:
            si = min(range(len(self.sides)), key=lambda i: sflops[i])
        else:
            si = self._wg_next % len(self.sides)  # round-robin (FLOP-balanced for every block measured no better)
            self._wg_next += 1
        side = self.sides[si]
        plan.wait_stream(side, torch.cuda.current_stream(self.device))
        f0 = K.FLOPS_ISSUED
        try:
            with torch.cuda.stream(side):
                yield
        finally:
            K.PHASE = prev
        sflops[si] += K.FLOPS_ISSUED - f0
        self.wg_event = torch.cuda.Event()
        plan.record_event(self.wg_event, side)

    _group_wg = True  # engines whose backward loop does not flush per block (VQVAETrainEngine) set False
    wg_balance = os.environ.get("SDMI_WG_FLUSH_BALANCE", "1") != "0"  # A/B switch of the flush-group stream choice

    def _grouping(self):
        return self._group_wg and self.side is not None

    def _wgrad_linear(self, dy, x, gW, gb=None):
        """A linear / 1x1-conv weight gradient (dW = dy^T x, db = column sums of dy) on the side stream. Grouped
        (default): deferred to the end of its block's backward (tape label) and issued there together with the
        block's other same-shape ones as ONE launch (K.linear_wgrad_grouped: one grid, one split-K reducer) -- e.g. a
        32^2 down block's self-attention out_proj, cross-attention q_proj and out_proj of both layers, six
        [384 x 384] x 32768 launches (and six reducers) before."""
        if not self._grouping():
            with self._wg(dy, x):
                K.linear_wgrad(dy, x, gW, bias_grad=gb)
            return
        self._keep.extend([dy, x])
        key = (tuple(dy.shape), K.ld_of(dy), tuple(x.shape), K.ld_of(x), gb is not None, gW.stride(0))
        self._pending_wg.setdefault(key, []).append((dy, x, gW, gb))

    def _flush_wg(self):
        """Issue the deferred weight gradients (groups of at most SDMI_GEMM_GROUP_MAX = 8) and the block's deferred
        GroupNorm dgamma / dbeta sums."""
        pend, self._pending_wg = self._pending_wg, {}
        # largest groups first, each on the side stream with less work issued so far: at the end of the backward the
        # last block's grouped launches are the tail the optimizer waits for (round 5: two ~160 us launches of the
        # 32^2 down block had both landed on one stream by round-robin parity while the other went idle)
        groups = [items[i:i + 8] for items in pend.values() for i in range(0, len(items), 8)]
        groups.sort(key=lambda g: -g[0][0].shape[0] * g[0][0].shape[1] * g[0][1].shape[1] * len(g))
        for grp in groups:
            with self._wg(balance=self.wg_balance):
                K.linear_wgrad_grouped(grp)
        gpend, self._pending_gn = self._pending_gn, []
        if gpend:
            # on the first weight-gradient stream, outside the round-robin (the block's other assignments unchanged)
            side = self.sides[0]
            plan.wait_stream(side, torch.cuda.current_stream(self.device))
            self._keep.extend(g[0] for g in gpend)
            with torch.cuda.stream(side):
                K.gn_rows_sum_grouped(gpend)

    _pending_wg = {}
    _pending_gn = []
    _time_inputs = []

    def _note_time_input(self):
        """The side-stream block just issued writes an input of the time-MLP backward (dtemb_all / dcp_all)."""
        if self.side is not None:
            self._time_inputs.append(self.wg_event)

    def _gn_defer(self):
        """GroupNorm backward dgamma / dbeta: summed over the batch on a weight-gradient stream at the block's flush
        (kernels.gn_bwd(defer=...)) -- the data-gradient chain then carries no batch tail per GroupNorm. Same-box A/B
        of the cond-UNet step: 13.55 / 13.49 ms inline, 13.37 / 13.34 ms deferred."""
        return self._pending_gn if self._grouping() else None

    def _join(self):
        """The current stream waits for all weight-gradient work issued so far."""
        if self.side is None:  # inline weight gradients (single-stream graph capture)
            return
        for side in self.sides:
            plan.wait_stream(torch.cuda.current_stream(self.device), side)

    # ------------------------------------------------------------------------------------------
    def backward(self, ctx, dpred, grads=None, on_progress=None):
        """dpred: NHWC bf16 [B*H*W, 8] (zero in padded channels). Writes every parameter gradient into
        `grads` ({key: fp32 view}, default: the engine's own) -- each is fully overwritten. on_progress(tape, k) runs
        after tape entry k (going backwards) and, at a block's end, its grouped weight gradients have been issued."""
        tape = ctx["tape"]
        for k in self.backward_steps(ctx, dpred, grads):
            if on_progress is not None:
                on_progress(tape, k)

    def backward_steps(self, ctx, dpred, grads=None):
        """The backward as a generator: yields tape position k once entry k (and, when it ends a block, the block's
        grouped weight gradients) has been issued; the final flush / side-stream join run when it is exhausted. The
        module path drives it segment by segment from several autograd nodes (sdmi.module_glue.StagedBackward)."""
        if grads is not None:
            self.Gd = grads
        assert self.Gd is not None, "engine built without gradient buffers"
        st = ctx["st"]
        B = st["B"]
        self.dpred = dpred
        self.dtemb_all = self._new(B, self.temb_total)
        self.temb_grad_all = self._temb_grad_view()
        self.dcp_all = self._new(B * st["S"], self.ctx_total) if st.get("ctx") is not None else None
        if self.dcp_all is not None:
            self._keep.append(self.dcp_all)  # written by side-stream dgrads, read by the final GEMM
        grads = ctx["grads"]
        tape = ctx["tape"]
        self._need_all()  # the optimizer chunks read the gradient buffers the backward is about to overwrite
        self._wg_next = 0  # same side-stream assignment every step
        self._side_flops = [0.0] * len(self.sides)
        K.PHASE = "bwd"
        self._pending_wg = {}
        self._pending_gn = []
        self._time_inputs = []
        for k in range(len(tape) - 1, -1, -1):
            fn, c = tape[k]
            fn(c, grads)
            if (self._pending_wg or self._pending_gn) and (k == 0 or tape[k - 1][1].get("label") != c.get("label")):
                self._flush_wg()  # the block's grouped weight gradients, before its gradients are reported final
            yield k
        self._flush_wg()
        self._join()
        self._keep = []
        self.dpred = None
        K.PHASE = ""

    # an attention block's input gradient reuses its output-gradient buffer (the GroupNorm backward then rewrites dy in
    # place, so the main stream first waits for the side-stream weight gradient reading dy)
    _dy_alias = True

    def _ctx_grad_view(self):
        """The context_proj weight gradients are one contiguous [sum C][ctx_dim] region of the flat store."""
        return contiguous_run(self.Gd, [f"{p}.context_proj.{l}.weight" for (p, l, c) in self._cross_layers()],
                              (self.ctx_total, self.L["ctx_dim"]))

    def _temb_grad_view(self):
        """The t_emb_layers weight gradients are one contiguous [sum C][T] region of the flat store."""
        return contiguous_run(self.Gd, [f"{p}.t_emb_layers.{l}.1.weight" for (p, l, ci, co) in self.resnets],
                              (self.temb_total, self.L["T"]))


class _WaitingParams(dict):
    """The engine's parameter dict: reading a parameter first makes the current stream wait for the optimizer
    chunk that updates it (when one is pending)."""

    def __init__(self, params, eng):
        super().__init__(params)
        self._eng = eng

    def __getitem__(self, k):
        eng = self._eng
        if eng._pending:
            eng._need(eng._key_chunk.get(k, 0))
        return dict.__getitem__(self, k)

    def raw(self, k):
        return dict.__getitem__(self, k)


def contiguous_run(tensors, keys, shape):
    """View over tensors[keys[0]] .. tensors[keys[-1]] that must lie back to back in memory."""
    first = tensors[keys[0]]
    pos = first.data_ptr()
    for k in keys:
        t = tensors[k]
        if t.data_ptr() != pos or not t.is_contiguous():
            raise RuntimeError(f"{k} is not contiguous with the previous tensors of its run (use sdmi.store.FlatStore)")
        pos += t.numel() * t.element_size()
    return first.as_strided(shape, torch.empty(shape, device="meta").stride())
