"""Explicit forward/backward schedule of the reference DiT (models/transformer.py:153-213,
transformer_layer.py:80-106, attention.py:33-78, multihead_attention.py:41-126, patch_embed.py:75-96) on the
HIP kernels of libsdmi.so, planned for MI355X:

  * tokens are row-major bf16 [B*N][D]; every Linear is one MFMA GEMM with bias / ReLU / position-embedding
    epilogues (the patch embedding is an implicit-GEMM 2x2 stride-2 convolution over the NHWC input, so the
    patchify rearrange never materialises);
  * the adaLN modulation of ALL layers plus the final norm is ONE GEMM ([B, 6*D*L + 2*D]) -- every layer's
    adaptive_norm_layer reads the same ReLU(t_emb); its backward is likewise one weight-gradient GEMM;
  * each gated residual add is fused into the LayerNorm+modulation kernel of the sub-block that follows it,
    and each gate backward into the LayerNorm backward that reads the same rows; the per-(sample, channel)
    gradients of shift / scale / gate are written as token-chunk partials and reduced once (no atomics);
  * self attention (9 heads x 32) and the optional text cross attention use the fused flash kernels.
Parameters are referenced by the reference's state-dict keys; gradients go to caller-owned fp32 views.
"""
import contextlib
import os

import torch

from . import _lib
from . import kernels as K
from . import streams
from . import plan
from .unet_engine import PackPlan, UNetEngine, _WaitingParams, contiguous_run


def dit_layout(cfg, im_channels=4):
    cond = cfg.get("condition_config") or {}
    types = cond.get("condition_types", []) if cond else []
    L = dict(D=cfg["hidden_size"], p=cfg["patch_size"], T=cfg["timestep_emb_dim"], n_layers=cfg["num_layers"],
             heads=cfg["num_heads"], head_dim=cfg["head_dim"], text="text" in types, image="image" in types,
             klass="class" in types, im_channels=im_channels)
    L["A"] = L["heads"] * L["head_dim"]
    if L["text"]:
        L["ctx_dim"] = cond["text_condition_config"]["text_embed_dim"]
    if L["image"]:
        ic = cond["image_condition_config"]
        L["im_in"] = ic["image_condition_input_channels"]
        L["im_out"] = ic["image_condition_output_channels"]
    if L["klass"]:
        L["num_classes"] = cond["class_condition_config"]["num_classes"]
    L["patch_in"] = im_channels + (L["im_out"] if L["image"] else 0)
    L["mod_w"] = 6 * L["D"] * L["n_layers"] + 2 * L["D"]
    return L


def ada_keys(L, what):
    return [f"transformer_layers.{i}.adaptive_norm_layer.1.{what}" for i in range(L["n_layers"])] + \
        [f"adaptive_norm_layer.1.{what}"]


def dit_flat_order(cfg, keys):
    """Flat-store order = order in which the backward finalises gradients: proj_out, layers last to first,
    then the adaLN weights (contiguous, one GEMM) and biases, then t_proj / patch embedding / conditioning."""
    L = dit_layout(cfg)
    aw, ab = ada_keys(L, "weight"), ada_keys(L, "bias")
    special = set(aw) | set(ab)
    head = [k for k in keys if k.startswith("proj_out")]
    layers = []
    for i in reversed(range(L["n_layers"])):
        pre = f"transformer_layers.{i}."
        lk = [k for k in keys if k.startswith(pre) and k not in special]
        vb = pre + "cross_attn_block.v_proj.bias"
        if vb in lk:  # k/v biases back to back: the packed k|v projection reads them as one vector
            lk.remove(vb)
            lk.insert(lk.index(pre + "cross_attn_block.k_proj.bias") + 1, vb)
        layers += lk
    tail = [k for k in keys if k not in special and k not in head and k not in layers]
    return head + layers + aw + ab + tail


def position_embedding(D, gh, gw):
    """2-D sin/cos table of models/patch_embed.py:5-34, computed once on the host in fp32 exactly as the
    reference does, cast to bf16 (the reference adds pos_embed.to(out.dtype), patch_embed.py:95)."""
    gy, gx = torch.meshgrid(torch.arange(gh, dtype=torch.float32), torch.arange(gw, dtype=torch.float32),
                            indexing="ij")
    gy, gx = gy.reshape(-1), gx.reshape(-1)
    q = D // 4
    factor = 10000 ** (torch.arange(0, q, dtype=torch.float32) / q)
    ey, ex = gy[:, None].repeat(1, q) / factor, gx[:, None].repeat(1, q) / factor
    return torch.cat([torch.sin(ey), torch.cos(ey), torch.sin(ex), torch.cos(ex)], dim=-1)


class DiTEngine:
    EPS = 1e-6  # nn.LayerNorm(..., eps=1E-6), transformer_layer.py:27,30; transformer.py:137

    def __init__(self, cfg, params, grads=None, im_channels=4, single_stream=False):
        self.cfg = cfg
        self.L = dit_layout(cfg, im_channels)
        L = self.L
        # class conditioning (transformer.py:176-181): sinusoidal t_emb += class @ class_emb.weight before t_proj,
        # one GEMM with the class count zero-padded to a multiple of 8
        self.kpad = (L["num_classes"] + 7) // 8 * 8 if L["klass"] else 0
        if L["D"] % 8 or L["D"] > 512 or L["D"] % 4:
            raise ValueError("hidden_size must be a multiple of 8 and <= 512 for the row kernels")
        if L["A"] % 8 or L["head_dim"] % 8 or L["head_dim"] > 64:
            raise ValueError("attention head_dim must be a multiple of 8 and <= 64")
        if L["text"] and (L["D"] // L["heads"]) % 8:
            raise ValueError("cross-attention head dim (hidden_size / num_heads) must be a multiple of 8")
        # optimizer / pack pipeline (trainer): chunk -> event the current stream still has to wait for before it reads
        # the chunk's parameters or packed weights (same protocol as the UNet engine)
        self._pending = {}
        self._key_chunk = {}
        self.P = _WaitingParams(params, self)
        self.Gd = grads
        self.im_channels = im_channels
        self.device = next(iter(params.values())).device
        # residual stream (and its gradient) dtype, read per engine: fp32 (default), or bf16 as the reference's autocast
        # keeps it (SDMI_DIT_STREAM=bf16; Model_DiT_12L_train.py:281-283, 345) -- a DIAGNOSTIC only: with the bf16 stream
        # the DiT-12L forward misses the north star's MSE <= 1e-4 against the fp32 reference
        self.SDT = torch.bfloat16 if os.environ.get("SDMI_DIT_STREAM", "fp32") == "bf16" else torch.float32
        # weight-gradient GEMMs of the backward run round-robin on side streams, overlapped with the data-gradient
        # chain on the current stream: one side stream (measured 0 / 1 / 2 / 3 streams -> 4.47 / 4.00 / 4.08 / 4.11 ms/step)
        self.sides = [streams.new_stream(self.device)] if self.device.type == "cuda" and not single_stream else []
        self.side = self.sides[0] if self.sides else None
        self._wg_next = 0
        self._keep = []
        self.cpad = (L["patch_in"] + 7) // 8 * 8
        self._pos = {}
        self.dgrad_t = True  # linear data gradients from transposed packs (3.5 % faster step)
        self._build_pack()

    # ------------------------------------------------------------------------------------------
    def _build_pack(self):
        P, L = self.P, self.L
        D, p = L["D"], L["p"]
        pk = PackPlan(self.device)

        def lin(key, name=None, t=False):
            w = P[key]
            N, Kd = w.shape
            pk.add(name or key, w, N, Kd, Kd, 1, 1, Kd, 1, 0, 0)
            if t and self.dgrad_t:  # [Kd][N] for the data gradient (B_NK GEMM)
                pk.add_transpose((name or key) + "#t", name or key, N, Kd, 1, [0], 8)

        # patch embedding Linear (D, (ph pw c)) as a 2x2 stride-2 conv weight [D][ph][pw][cpad]
        w = P["patch_embed_layer.patch_embed.0.weight"]
        ci = L["patch_in"]
        pk.add("pe", w, D, ci, self.cpad, p, p, p * p * ci, 1, p * ci, ci)
        lin("t_proj.0.weight")
        lin("t_proj.2.weight")
        if L["klass"]:  # [classes (zero rows up to kpad)][T]: B operand (k = class) of the class-embedding GEMM
            pk.add("class_emb#kn", P["class_emb.weight"], L["num_classes"], L["T"], L["T"], 1, 1, L["T"], 1, 0, 0,
                   rows=self.kpad)
        pk.reserve("ada", L["mod_w"], D)
        row = 0
        for k in ada_keys(L, "weight"):
            wk = P[k]
            pk.add(None, wk, wk.shape[0], D, D, 1, 1, D, 1, 0, 0, into="ada", row0=row)
            row += wk.shape[0]
        for i in range(L["n_layers"]):
            q = f"transformer_layers.{i}."
            lin(q + "attn_block.qkv_proj.weight", t=True)
            lin(q + "attn_block.output_proj.0.weight", t=True)
            lin(q + "mlp_block.0.weight", t=True)
            lin(q + "mlp_block.2.weight", t=True)
            if L["text"]:
                lin(q + "cross_attn_block.q_proj.weight", t=True)
                lin(q + "cross_attn_block.out_proj.weight", t=True)
                lin(q + "context_proj.weight")
                pk.reserve(q + "kv", 2 * D, D)
                pk.add(None, P[q + "cross_attn_block.k_proj.weight"], D, D, D, 1, 1, D, 1, 0, 0, into=q + "kv")
                pk.add(None, P[q + "cross_attn_block.v_proj.weight"], D, D, D, 1, 1, D, 1, 0, 0, into=q + "kv",
                       row0=D)
                if self.dgrad_t:
                    pk.add_transpose(q + "kv#t", q + "kv", 2 * D, D, 1, [0], 8)
        lin("proj_out.weight")
        pk.finalize()
        self.pack = pk

    def _dgrad(self, dy, key, out, **kw):
        """Data gradient of the packed linear `key` ([N][K]): from its transposed copy key#t when packed."""
        if self.dgrad_t:
            K.linear_dgrad_t(dy, self.W(key + "#t"), out, **kw)
        else:
            K.linear_dgrad(dy, self.W(key), out, **kw)

    def kv_bias(self, i):
        """k_proj.bias | v_proj.bias of layer i: adjacent in the flat store (dit_flat_order)."""
        q = f"transformer_layers.{i}.cross_attn_block."
        return contiguous_run(self.P, [q + "k_proj.bias", q + "v_proj.bias"], (2 * self.L["D"],))

    def W(self, name):
        if self._pending:
            self._need(self.pack.view_chunk.get(name, 0))
        return self.pack.view(name)

    # forward-ordered optimizer chunks (sdmi.trainer): the UNet engine's protocol
    set_chunks = UNetEngine.set_chunks
    _need = UNetEngine._need
    _need_all = UNetEngine._need_all

    refresh_weights = UNetEngine.refresh_weights

    def pos_table(self, gh, gw):
        key = (gh, gw)
        if key not in self._pos:
            self._pos[key] = position_embedding(self.L["D"], gh, gw).to(torch.bfloat16).to(self.device)
        return self._pos[key]


    def _new(self, rows, C, dtype=torch.bfloat16):
        return torch.empty(rows, C, dtype=dtype, device=self.device)

    def g(self, key):
        return self.Gd[key] if self.Gd is not None else None

    # ------------------------------------------------------------------------------------------
    def _ln_fwd(self, x, y, mean, rstd, *, v=None, gate=None, xo=None, shift=None, scale=None, N):
        mod = shift if shift is not None else gate
        ld_mod = K.ld_of(mod) if mod is not None else 0
        _lib.check(_lib.lib().sdmi_ln_mod_fwd(
            x.data_ptr(), K.ld_of(x), K._p(v), K.ld_of(v) if v is not None else 0, K._p(gate), K._p(xo),
            K.ld_of(xo) if xo is not None else 0, K._p(shift), K._p(scale), ld_mod, y.data_ptr(), K.ld_of(y),
            mean.data_ptr(), rstd.data_ptr(), x.shape[0], x.shape[1], N, self.EPS, int(x.dtype == torch.float32),
            K._stream()), "sdmi_ln_mod_fwd")

    def _ln_bwd(self, x, mean, rstd, dy, dx, *, scale=None, dres=None, psh=None, psc=None, gate=None, v=None,
                dv=None, pg=None, dx16=None, N):
        mod = scale if scale is not None else gate
        ld_mod = K.ld_of(mod) if mod is not None else 0
        ws_ld = self.ws.shape[1]
        _lib.check(_lib.lib().sdmi_ln_mod_bwd(
            x.data_ptr(), K.ld_of(x), mean.data_ptr(), rstd.data_ptr(), dy.data_ptr(), K.ld_of(dy), K._p(scale),
            ld_mod, K._p(dres), K.ld_of(dres) if dres is not None else 0, dx.data_ptr(), K.ld_of(dx), K._p(psh),
            K._p(psc), ws_ld, K._p(gate), K._p(v), K.ld_of(v) if v is not None else 0, K._p(dv),
            K.ld_of(dv) if dv is not None else 0, K._p(pg), x.shape[0], x.shape[1], N, int(x.dtype == torch.float32),
            K._p(dx16), K.ld_of(dx16) if dx16 is not None else 0, K._stream()), "sdmi_ln_mod_bwd")

    def forward(self, x, t, text=None, mask=None, need_backward=True, mask_keep=None, klass=None):
        """x: (B, C, H, W) fp32; t: int64 (B,), (1,) or 0-d; text (B, S, ctx); mask (B, cmi, MH, MW) fp32;
        klass (B, num_classes) fp32 for class-conditional configs.
        Returns (pred fp32 token-major [B*N, p*p*C], ctx for backward)."""
        L, P = self.L, self.P
        B, Cx, H, W = x.shape
        assert Cx == self.im_channels
        D, p, Hh, hd, A = L["D"], L["p"], L["heads"], L["head_dim"], L["A"]
        if H % p or W % p:
            raise ValueError("input height / width must be divisible by the patch size")
        gh, gw = H // p, W // p
        N = gh * gw
        M = B * N
        x = plan.as_operand(x)
        st = dict(B=B, H=H, W=W, N=N, M=M)
        # ---- patch source (transformer.py:180-188) + patch embedding (patch_embed.py:75-96) ----
        xin = self._new(B * H * W, self.cpad)
        m = (plan.as_operand(mask, torch.uint8 if K.is_class_map(mask) else torch.float32) if L["image"] else None)
        K.prep_input(x, B, Cx, H, W, m, L.get("im_in", 0), P["cond_conv_in.weight"] if m is not None else None,
                     L.get("im_out", 0),
                     xin, self.cpad, mask_keep)
        st.update(xin=xin, mask=m, keep=mask_keep)
        # the residual stream is self.SDT: fp32 by default (the reference's autocast stream is bf16; fp32 is strictly
        # closer to its fp32 forward and costs only row-kernel bandwidth -- the stream is never a GEMM operand)
        tok = self._new(M, D, self.SDT)
        g = K.conv_geom(H, W, self.cpad, self.cpad, p, p, gh, gw, p, p, 0, 0)
        K.gemm(M, D, p * p * self.cpad, xin, _lib.A_CONV, 0, self.W("pe"), _lib.B_NK, p * p * self.cpad, tok, D,
               geom=g, bias=P["patch_embed_layer.patch_embed.0.bias"], rowbias=self.pos_table(gh, gw), rb_ld=D,
               rb_div=1, rb_mod=N)
        # ---- time embedding -> t_proj (ReLU) -> ReLU(t_emb) -> all adaLN tables in one GEMM ----
        t = plan.timesteps(t, self.device)
        if t.numel() not in (1, B):
            raise ValueError("t must have 1 or B elements")
        e = self._new(B, L["T"])
        _lib.check(_lib.lib().sdmi_time_embedding(t.data_ptr(), 0 if t.numel() == 1 else 1, B, L["T"], e.data_ptr(),
                                                  L["T"], None, K._stream()), "sdmi_time_embedding")
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
            K.gemm(B, L["T"], self.kpad, cls, _lib.A_ROWMAJOR, self.kpad, self.W("class_emb#kn"), _lib.B_KN, L["T"],
                   e, L["T"], resid=e, ldr=L["T"])  # e += class @ class_emb.weight
        h1 = self._new(B, D)
        K.linear(e, self.W("t_proj.0.weight"), h1, bias=P["t_proj.0.bias"], act=2)
        r = self._new(B, D)  # ReLU(t_emb): the only form in which t_emb is consumed (adaLN inputs)
        K.linear(h1, self.W("t_proj.2.weight"), r, bias=P["t_proj.2.bias"], act=2)
        mod = self._new(B, L["mod_w"])
        ada_b = contiguous_run(P, ada_keys(L, "bias"), (L["mod_w"],))
        K.linear(r, self.W("ada"), mod, bias=ada_b)
        st.update(e=e, h1=h1, r=r, mod=mod, cls=cls)
        ctx = None
        if L["text"]:
            txt = plan.as_operand(text)
            S = txt.shape[1]
            ctx = self._new(B * S, txt.shape[2])
            _lib.check(_lib.lib().sdmi_nchw_to_nhwc_bf16(txt.data_ptr(), B * S, txt.shape[2], 1, ctx.data_ptr(),
                                                         txt.shape[2], K._stream()), "cast")
            st["S"] = S
        st["ctx"] = ctx

        def mcol(i, j):
            o = 6 * D * i + j * D
            return mod[:, o:o + D]

        layers = []
        xs, pend = tok, None  # residual stream, pending gated branch (v, gate) to add before the next norm
        for i in range(L["n_layers"]):
            q = f"transformer_layers.{i}."
            c = dict(i=i)
            y1, m1, r1 = self._new(M, D), self._new(M, 1, torch.float32), self._new(M, 1, torch.float32)
            if pend is None:
                xl = xs
                self._ln_fwd(xs, y1, m1, r1, shift=mcol(i, 0), scale=mcol(i, 1), N=N)
            else:
                xl = self._new(M, D, self.SDT)
                self._ln_fwd(xs, y1, m1, r1, v=pend[0], gate=pend[1], xo=xl, shift=mcol(i, 0), scale=mcol(i, 1), N=N)
            qkv = self._new(M, 3 * A)
            K.linear(y1, self.W(q + "attn_block.qkv_proj.weight"), qkv, bias=P[q + "attn_block.qkv_proj.bias"])
            o = self._new(M, A)
            lse = K.attn_fwd(qkv[:, :A], qkv[:, A:2 * A], qkv[:, 2 * A:], o, B, Hh, N, N, hd)
            v1 = self._new(M, D)
            K.linear(o, self.W(q + "attn_block.output_proj.0.weight"), v1, bias=P[q + "attn_block.output_proj.0.bias"])
            c.update(xl=xl, y1=y1, m1=m1, r1=r1, qkv=qkv, o=o, lse=lse, v1=v1)
            x2, y2 = self._new(M, D, self.SDT), self._new(M, D)
            m2, r2 = self._new(M, 1, torch.float32), self._new(M, 1, torch.float32)
            if L["text"]:
                # out = x + gate*attn ; out = out + cross_attn(LN(out), ctx_proj) (ungated, transformer_layer.py:93-102)
                xc, yc = self._new(M, D, self.SDT), self._new(M, D)
                mc, rc = self._new(M, 1, torch.float32), self._new(M, 1, torch.float32)
                self._ln_fwd(xl, yc, mc, rc, v=v1, gate=mcol(i, 2), xo=xc, N=N)
                S = st["S"]
                cq = self._new(M, D)
                K.linear(yc, self.W(q + "cross_attn_block.q_proj.weight"), cq, bias=P[q + "cross_attn_block.q_proj.bias"])
                cp = self._new(B * S, D)
                K.linear(ctx, self.W(q + "context_proj.weight"), cp, bias=P[q + "context_proj.bias"])
                ckv = self._new(B * S, 2 * D)
                K.linear(cp, self.W(q + "kv"), ckv, bias=self.kv_bias(i))
                co = self._new(M, D)
                clse = K.attn_fwd(cq, ckv[:, :D], ckv[:, D:], co, B, Hh, N, S, D // Hh)
                vc = self._new(M, D)
                K.linear(co, self.W(q + "cross_attn_block.out_proj.weight"), vc,
                         bias=P[q + "cross_attn_block.out_proj.bias"])
                self._ln_fwd(xc, y2, m2, r2, v=vc, xo=x2, shift=mcol(i, 3), scale=mcol(i, 4), N=N)
                c.update(xc=xc, yc=yc, mc=mc, rc=rc, cq=cq, cp=cp, ckv=ckv, co=co, clse=clse)
            else:
                self._ln_fwd(xl, y2, m2, r2, v=v1, gate=mcol(i, 2), xo=x2, shift=mcol(i, 3), scale=mcol(i, 4), N=N)
            hbuf = self._new(M, 4 * D)
            K.linear(y2, self.W(q + "mlp_block.0.weight"), hbuf, bias=P[q + "mlp_block.0.bias"], act=2)
            v2 = self._new(M, D)
            K.linear(hbuf, self.W(q + "mlp_block.2.weight"), v2, bias=P[q + "mlp_block.2.bias"])
            c.update(x2=x2, y2=y2, m2=m2, r2=r2, h=hbuf, v2=v2)
            layers.append(c)
            xs, pend = x2, (v2, mcol(i, 5))
        # ---- final adaLN-modulated norm + proj_out (transformer.py:203-207) ----
        of = 6 * D * L["n_layers"]
        xf, yf = self._new(M, D, self.SDT), self._new(M, D)
        mf, rf = self._new(M, 1, torch.float32), self._new(M, 1, torch.float32)
        self._ln_fwd(xs, yf, mf, rf, v=pend[0], gate=pend[1], xo=xf, shift=mod[:, of:of + D],
                     scale=mod[:, of + D:of + 2 * D], N=N)
        npo = p * p * self.im_channels
        pred = self._new(M, npo, torch.float32)
        K.linear(yf, self.W("proj_out.weight"), pred, bias=P["proj_out.bias"])
        st.update(xf=xf, yf=yf, mf=mf, rf=rf, layers=layers)
        return pred, (dict(st=st) if need_backward else None)

    # ------------------------------------------------------------------------------------------
    def loss(self, pred, noise, dpred, loss_out, gscale_dev=None, gscale=1.0):
        """nn.MSELoss(pred, noise) read straight from the token layout; dpred (bf16, same layout) = dL/dpred."""
        B, C, H, W = noise.shape
        ws = torch.empty(_lib.lib().sdmi_mse_workspace() // 4, dtype=torch.float32, device=self.device)
        _lib.check(_lib.lib().sdmi_mse_patch(pred.data_ptr(), pred.shape[1], noise.data_ptr(), B, C, H, W, self.L["p"],
                                             gscale, K._p(gscale_dev), K._p(dpred), ws.data_ptr(), loss_out.data_ptr(),
                                             K._stream()), "sdmi_mse_patch")

    def pred_to_nchw(self, pred, B, H, W):
        out = torch.empty(B, self.im_channels, H, W, dtype=torch.float32, device=self.device)
        _lib.check(_lib.lib().sdmi_tokens_to_nchw(pred.data_ptr(), 1, pred.shape[1], B, self.im_channels, H, W,
                                                  self.L["p"], out.data_ptr(), K._stream()), "sdmi_tokens_to_nchw")
        return out

    def dpred_from_nchw(self, d):
        B, C, H, W = d.shape
        p = self.L["p"]
        dp = self._new(B * (H // p) * (W // p), p * p * C)
        _lib.check(_lib.lib().sdmi_nchw_to_tokens_bf16(d.data_ptr(), B, C, H, W, p, dp.data_ptr(), p * p * C,
                                                       K._stream()), "sdmi_nchw_to_tokens_bf16")
        return dp

    def new_dpred(self, B, H, W):
        p = self.L["p"]
        return self._new(B * (H // p) * (W // p), p * p * self.im_channels)

    # ------------------------------------------------------------------------------------------
    @contextlib.contextmanager
    def _wg(self, *keep):
        """Weight-gradient work on the next side stream, after everything issued so far on the current stream;
        `keep` pins its operands until the backward's final join (the allocator must not hand their memory to the
        current stream while a side stream still reads it)."""
        if self.side is None or not self.sides:  # inline (single-stream graph capture)
            yield
            return
        self._keep.extend(keep)
        side = self.sides[self._wg_next % len(self.sides)]
        self._wg_next += 1
        plan.wait_stream(side, torch.cuda.current_stream(self.device))
        with torch.cuda.stream(side):
            yield

    # the projections' weight gradients of consecutive layers go out as one launch per shape, in groups of 7, 3 and 2
    # layers from the last layer down: the group issued after the final layer's backward is the tail the step waits
    # for, so it is kept short. Measured DiT-12L step, same box, uniform groups of 1 / 3 / 6 layers: 4.44 / 4.11 / 4.04
    # ms (round 3); 6+6 3.66 / 3.66, 6+4+2 3.58 / 3.57, 7+3+2 3.56 / 3.55, 5+4+2+1 3.62, 6+4+1+1 3.63 ms (round 4)
    # Any depth: a short 3 + 2 tail and groups of at most 7 layers before it, evened out (12 layers: 7, 3, 2; 28 layers:
    # 6, 6, 6, 5, 3, 2), so a deeper DiT keeps issuing weight gradients (and DP buckets / norm pieces) as it goes.
    _pending_wg = {}

    @staticmethod
    def dit_groups(n_layers):
        if n_layers <= 5:
            return (n_layers,)
        head = n_layers - 5
        k = -(-head // 7)
        return tuple(head // k + (1 if i < head % k else 0) for i in range(k)) + (3, 2)

    @property
    def _dit_groups(self):
        return self.dit_groups(self.L["n_layers"])

    def _flush_after(self, n_done):
        """True when the grouped weight gradients are issued after the backward of n_done layers."""
        acc = 0
        for g in self._dit_groups:
            acc += g
            if n_done == acc:
                return True
        return n_done == self.L["n_layers"]

    def _wgrad_linear(self, dy, x, gW, gb=None):
        """dW = dy^T x (+ db) on a side stream; deferred and grouped by shape (UNetEngine._wgrad_linear)."""
        if max(self._dit_groups) <= 1 or self.side is None:
            with self._wg(dy, x):
                K.linear_wgrad(dy, x, gW, bias_grad=gb)
            return
        self._keep.extend([dy, x])
        key = (tuple(dy.shape), K.ld_of(dy), tuple(x.shape), K.ld_of(x), gb is not None, gW.stride(0))
        self._pending_wg.setdefault(key, []).append((dy, x, gW, gb))

    def _flush_wg(self):
        pend, self._pending_wg = self._pending_wg, {}
        for items in pend.values():
            for j in range(0, len(items), 8):
                with self._wg():
                    K.linear_wgrad_grouped(items[j:j + 8])

    def _join(self):
        """The current stream waits for all weight-gradient work issued so far."""
        if self.side is None:
            return
        for side in self.sides:
            plan.wait_stream(torch.cuda.current_stream(self.device), side)

    def backward(self, ctx, dpred, grads=None, on_progress=None):
        """dpred: bf16 token-major [B*N, p*p*C]. Writes every parameter gradient (fully overwritten). on_progress(i)
        runs once layer i's gradients (and proj_out's) have all been issued."""
        for i in self.backward_steps(ctx, dpred, grads):
            if on_progress is not None:
                on_progress(i)

    def backward_steps(self, ctx, dpred, grads=None):
        """The backward as a generator: yields layer index i once layers i..L-1 and proj_out are final (their grouped
        weight gradients issued); the adaLN / t_proj / patch-embedding tail and the side-stream join run when it is
        exhausted (sdmi.module_glue.StagedBackward drives it segment by segment)."""
        if grads is not None:
            self.Gd = grads
        assert self.Gd is not None, "engine built without gradient buffers"
        self._need_all()  # the optimizer chunks read the gradient buffers the backward is about to overwrite
        self._wg_next = 0
        self._pending_wg = {}
        L, P = self.L, self.P
        st = ctx["st"]
        B, H, W, N, M = st["B"], st["H"], st["W"], st["N"], st["M"]
        D, p, Hh, hd, A = L["D"], L["p"], L["heads"], L["head_dim"], L["A"]
        mod = st["mod"]
        R = _lib.lib().sdmi_ln_chunk_rows(N)
        chunks = N // R
        # partial rows of the modulation gradient: [(b, chunk)][mod_w]; every column is written exactly once
        self.ws = torch.empty(B * chunks, L["mod_w"], dtype=torch.float32, device=self.device)
        ws = self.ws

        def mcol(t, i, j):
            o = 6 * D * i + j * D
            return t[:, o:o + D]

        # ---- proj_out + final norm ----
        with self._wg(dpred, st["yf"]):
            K.linear_wgrad(dpred, st["yf"], self.g("proj_out.weight"), bias_grad=self.g("proj_out.bias"))
        dy = self._new(M, D)
        K.linear_dgrad(dpred, self.W("proj_out.weight"), dy)
        of = 6 * D * L["n_layers"]
        dxs = self._new(M, D, self.SDT)  # gradient of the residual stream, updated in place
        dv2 = self._new(M, D)
        last = st["layers"][-1]
        self._ln_bwd(st["xf"], st["mf"], st["rf"], dy, dxs, scale=mod[:, of + D:of + 2 * D], psh=ws[:, of:],
                     psc=ws[:, of + D:], gate=mcol(mod, L["n_layers"] - 1, 5), v=last["v2"], dv=dv2,
                     pg=mcol(ws, L["n_layers"] - 1, 5), N=N)
        for i in reversed(range(L["n_layers"])):
            c = st["layers"][i]
            q = f"transformer_layers.{i}."
            # MLP (transformer_layer.py:104-106)
            self._wgrad_linear(dv2, c["h"], self.g(q + "mlp_block.2.weight"), self.g(q + "mlp_block.2.bias"))
            dh = self._new(M, 4 * D)
            self._dgrad(dv2, q + "mlp_block.2.weight", dh, relu_of=c["h"])
            self._wgrad_linear(dh, c["y2"], self.g(q + "mlp_block.0.weight"), self.g(q + "mlp_block.0.bias"))
            dy2 = self._new(M, D)
            self._dgrad(dh, q + "mlp_block.0.weight", dy2)
            dv1 = self._new(M, D)
            if L["text"]:
                # x2 = xc + cross(LN(xc)) ; y2 = LNmod(x2)
                dvc = self._new(M, D)  # bf16 copy of d(x2) = gradient of the ungated cross-attention branch
                self._ln_bwd(c["x2"], c["m2"], c["r2"], dy2, dxs, scale=mcol(mod, i, 4), dres=dxs,
                             psh=mcol(ws, i, 3), psc=mcol(ws, i, 4), dx16=dvc, N=N)
                S = st["S"]
                self._wgrad_linear(dvc, c["co"], self.g(q + "cross_attn_block.out_proj.weight"),
                                   self.g(q + "cross_attn_block.out_proj.bias"))
                dco = self._new(M, D)
                self._dgrad(dvc, q + "cross_attn_block.out_proj.weight", dco)
                dcq, dckv = self._new(M, D), self._new(B * S, 2 * D)
                K.attn_bwd(c["cq"], c["ckv"][:, :D], c["ckv"][:, D:], c["co"], dco, c["clse"], dcq, dckv[:, :D],
                           dckv[:, D:], B, Hh, N, S, D // Hh)
                self._wgrad_linear(dcq, c["yc"], self.g(q + "cross_attn_block.q_proj.weight"),
                                   self.g(q + "cross_attn_block.q_proj.bias"))
                self._wgrad_linear(dckv[:, :D], c["cp"], self.g(q + "cross_attn_block.k_proj.weight"),
                                   self.g(q + "cross_attn_block.k_proj.bias"))
                self._wgrad_linear(dckv[:, D:], c["cp"], self.g(q + "cross_attn_block.v_proj.weight"),
                                   self.g(q + "cross_attn_block.v_proj.bias"))
                dcp = self._new(B * S, D)
                self._dgrad(dckv, q + "kv", dcp)
                self._wgrad_linear(dcp, st["ctx"], self.g(q + "context_proj.weight"), self.g(q + "context_proj.bias"))
                dyc = self._new(M, D)
                self._dgrad(dcq, q + "cross_attn_block.q_proj.weight", dyc)
                self._ln_bwd(c["xc"], c["mc"], c["rc"], dyc, dxs, dres=dxs, gate=mcol(mod, i, 2), v=c["v1"], dv=dv1,
                             pg=mcol(ws, i, 2), N=N)
            else:
                self._ln_bwd(c["x2"], c["m2"], c["r2"], dy2, dxs, scale=mcol(mod, i, 4), dres=dxs, psh=mcol(ws, i, 3),
                             psc=mcol(ws, i, 4), gate=mcol(mod, i, 2), v=c["v1"], dv=dv1, pg=mcol(ws, i, 2), N=N)
            # self attention (attention.py:33-78)
            self._wgrad_linear(dv1, c["o"], self.g(q + "attn_block.output_proj.0.weight"),
                               self.g(q + "attn_block.output_proj.0.bias"))
            do = self._new(M, A)
            self._dgrad(dv1, q + "attn_block.output_proj.0.weight", do)
            qkv = c["qkv"]
            dqkv = self._new(M, 3 * A)
            K.attn_bwd(qkv[:, :A], qkv[:, A:2 * A], qkv[:, 2 * A:], c["o"], do, c["lse"], dqkv[:, :A],
                       dqkv[:, A:2 * A], dqkv[:, 2 * A:], B, Hh, N, N, hd)
            self._wgrad_linear(dqkv, c["y1"], self.g(q + "attn_block.qkv_proj.weight"),
                               self.g(q + "attn_block.qkv_proj.bias"))
            dy1 = self._new(M, D)
            self._dgrad(dqkv, q + "attn_block.qkv_proj.weight", dy1)
            prev = st["layers"][i - 1] if i > 0 else None
            dv2 = self._new(M, D) if prev is not None else None
            dtok = self._new(M, D) if prev is None else None  # bf16 d(tokens): patch-embedding GEMM operand
            self._ln_bwd(c["xl"], c["m1"], c["r1"], dy1, dxs, scale=mcol(mod, i, 1), dres=dxs, psh=mcol(ws, i, 0),
                         psc=mcol(ws, i, 1), gate=mcol(mod, i - 1, 5) if prev else None,
                         v=prev["v2"] if prev else None, dv=dv2, pg=mcol(ws, i - 1, 5) if prev else None, dx16=dtok,
                         N=N)
            # grouped weight gradients: issued after each group of _dit_groups layers (same-shape projections of those
            # layers in one launch each); the layers are reported final only once their gradients are issued
            if self._pending_wg and self._flush_after(L["n_layers"] - i):
                self._flush_wg()
            if not self._pending_wg:
                yield i
        self._flush_wg()
        # ---- adaLN tables of every layer: one reduction, one weight-gradient GEMM ----
        dmod = self._new(B, L["mod_w"])
        _lib.check(_lib.lib().sdmi_mod_finalize(ws.data_ptr(), B, chunks, L["mod_w"], L["mod_w"], dmod.data_ptr(),
                                                L["mod_w"], K._stream()), "sdmi_mod_finalize")
        with self._wg(dmod, st["r"]):
            K.linear_wgrad(dmod, st["r"], contiguous_run(self.Gd, ada_keys(L, "weight"), (L["mod_w"], D)),
                           bias_grad=contiguous_run(self.Gd, ada_keys(L, "bias"), (L["mod_w"],)))
        dt = self._new(B, D)
        K.linear_dgrad(dmod, self.W("ada"), dt, relu_of=st["r"])
        with self._wg(dt, st["h1"]):
            K.linear_wgrad(dt, st["h1"], self.g("t_proj.2.weight"), bias_grad=self.g("t_proj.2.bias"))
        dh1 = self._new(B, D)
        K.linear_dgrad(dt, self.W("t_proj.2.weight"), dh1, relu_of=st["h1"])
        with self._wg(dh1, st["e"]):
            K.linear_wgrad(dh1, st["e"], self.g("t_proj.0.weight"), bias_grad=self.g("t_proj.0.bias"))
        if st.get("cls") is not None:  # d class_emb.weight = class^T @ d(t_emb), d(t_emb) = dh1 @ W(t_proj.0)
            de = self._new(B, L["T"])
            K.linear_dgrad(dh1, self.W("t_proj.0.weight"), de)
            K.gemm(self.kpad, L["T"], B, st["cls"], _lib.A_COLMAJOR, self.kpad, de, _lib.B_KN, L["T"],
                   self.g("class_emb.weight"), L["T"], m_store=L["num_classes"])
        # ---- patch embedding (a 2x2 stride-2 conv over the NHWC patch source) ----
        gh, gw = H // p, W // p
        xin = st["xin"]
        K.conv_wgrad(dtok, D, xin, B, H, W, self.cpad, self.cpad, D, p, p, p, 0,
                     self.g("patch_embed_layer.patch_embed.0.weight"), gh, gw, perm=(self.cpad, p * p, L["patch_in"], 2),
                     bias_grad=self.g("patch_embed_layer.patch_embed.0.bias"))
        if L["image"]:
            # d(patch source): each input pixel feeds exactly one token -> p*p sub-pixel GEMMs [M, D] x [D, cpad]
            dxin = self._new(B * H * W, self.cpad)
            wpe = self.W("pe")
            for ph in range(p):
                for pw in range(p):
                    tap = ph * p + pw
                    remap = (gh, gw, H, W, p, p, ph, pw)
                    K.gemm(M, self.cpad, D, dtok, _lib.A_ROWMAJOR, D, wpe[:, tap * self.cpad:], _lib.B_KN,
                           p * p * self.cpad, dxin, self.cpad, remap=remap)
            K.cond_wgrad(dxin, self.cpad, self.im_channels, B, H, W, st["mask"], L["im_in"], L["im_out"],
                         self.g("cond_conv_in.weight"), st["keep"])
        self._join()
        self._keep = []
        self.ws = None
