"""VQVAE training step (the autoencoder stage of the reference: train_vqvae_celebhq.py:405-470, models/vqvae.py:93-158)
on the HIP kernels of libsdmi.so -- forward, reconstruction MSE + codebook / commitment losses, the straight-through
backward through decoder, quantiser and encoder, and Adam(betas=(0.5, 0.999)).

    encoder (conv_in -> DownBlocks -> MidBlocks -> GN+SiLU -> conv_out) -> pre_quant_conv -> nearest code (STE)
    -> post_quant_conv -> decoder (conv_in -> MidBlocks -> UpBlocks -> GN+SiLU -> conv_out)
    loss = MSE(out, im) + codebook_weight * mean((q - sg[x])^2) + commitment_beta * mean((sg[q] - x)^2)

The blocks are the UNet engine's (sdmi.unet_engine: same resnet / self-attention / stride-2 conv / transposed-conv
kernels and backward schedule, t_emb_dim=None so no time-embedding terms); the latent interface is two kernels:
sdmi_vq_quantize (pre_quant_conv + cdist/argmin + STE output, vqvae.py:93-126) and sdmi_vq_bwd (post_quant_conv
backward, straight-through gradient + commitment term, pre_quant_conv backward, the codebook rows' gradient).
LPIPS and the PatchGAN terms of the reference trainer are out of scope (LPIPS needs a pretrained VGG16
download); so is its fp32-only arithmetic: activations are bf16 here, accumulation fp32, master weights fp32."""
import torch
import torch.distributed as dist

from . import _lib
from . import kernels as K
from . import plan
from . import streams
from .store import FlatStore
from .unet_engine import Grads, PackPlan, Tape, UNetEngine
from .vqvae_engine import vqvae_layout

S_NORM, S_COEF, S_SCALE, S_GROWTH, S_STEP, S_SKIP, S_LOSS = range(7)


class VQVAETrainEngine(UNetEngine):
    """Forward + backward of models/vqvae.py VQVAE. Parameters / gradients: {state-dict key: fp32 CUDA tensor}."""

    _group_wg = False  # its own backward loop issues every weight gradient in place (no per-block grouping)

    def __init__(self, cfg, params, grads=None, im_channels=3):
        import os
        self.cfg = cfg
        self.L = vqvae_layout(cfg)
        L = self.L
        if L["z"] > 8:
            raise ValueError("z_channels > 8 is not supported by sdmi_vq_quantize")
        for c in L["down"] + L["mid"]:
            if c % 8:
                raise ValueError("channel counts must be multiples of 8")
        self.base = "vqvae"
        self.P = params
        self.Gd = grads
        self._pending, self._key_chunk = {}, {}
        self.im_channels = im_channels
        self.device = next(iter(params.values())).device
        self.cin_pad = (im_channels + 7) // 8 * 8
        self.temb_off = {}  # no time embedding anywhere (blocks built with t_emb_dim=None)
        self.temb_total = 0
        self.side = streams.new_stream(self.device) if self.device.type == "cuda" else None
        self.sides = [self.side] if self.side is not None else []  # the UNet engine's _wg / _join round-robin
        self._wg_next = 0
        self._keep = []
        self.dgrad_t = False
        self._build_pack()

    # ------------------------------------------------------------------------------------------
    def _resnets(self):
        L = self.L
        d, m = L["down"], L["mid"]
        out = []
        for i in range(len(d) - 1):
            out += [(f"encoder_layers.{i}", l, d[i] if l == 0 else d[i + 1], d[i + 1]) for l in range(L["n_down"])]
        for i in range(len(m) - 1):
            out += [(f"encoder_mids.{i}", l, m[i] if l == 0 else m[i + 1], m[i + 1]) for l in range(L["n_mid"] + 1)]
        for j, i in enumerate(reversed(range(1, len(m)))):
            out += [(f"decoder_mids.{j}", l, m[i] if l == 0 else m[i - 1], m[i - 1]) for l in range(L["n_mid"] + 1)]
        for j, i in enumerate(reversed(range(1, len(d)))):
            out += [(f"decoder_layers.{j}", l, d[i] if l == 0 else d[i - 1], d[i - 1]) for l in range(L["n_up"])]
        return out

    def _attn_keys(self):
        L = self.L
        d, m = L["down"], L["mid"]
        keys = []
        for i in range(len(d) - 1):
            if L["attn"][i]:
                keys += [f"encoder_layers.{i}.attentions.{l}" for l in range(L["n_down"])]
        for i in range(len(m) - 1):
            keys += [f"encoder_mids.{i}.attentions.{l}" for l in range(L["n_mid"])]
        for j in range(len(m) - 1):
            keys += [f"decoder_mids.{j}.attentions.{l}" for l in range(L["n_mid"])]
        for j, i in enumerate(reversed(range(1, len(d)))):
            if L["attn"][i - 1]:
                keys += [f"decoder_layers.{j}.attentions.{l}" for l in range(L["n_up"])]
        return keys

    def _build_pack(self):
        L = self.L
        pk = PackPlan(self.device)
        self._pk_conv(pk, "encoder_conv_in", dgrad=False, ipad=self.cin_pad)  # the image needs no gradient
        for (p, l, cin, cout) in self._resnets():
            self._pk_resnet(pk, p, l, cin, cout)
        for key in self._attn_keys():
            self._pk_lin(pk, key + ".in_proj_weight")
            self._pk_lin(pk, key + ".out_proj")
        d = L["down"]
        for i in range(len(d) - 1):
            if L["ds"][i]:
                self._pk_down(pk, f"encoder_layers.{i}.down_sample_conv")
        self._pk_conv(pk, "encoder_conv_out", opad=8)
        self._pk_conv(pk, "decoder_conv_in", ipad=8)
        for j, i in enumerate(reversed(range(1, len(d)))):
            if L["ds"][i - 1]:
                self._pk_up(pk, f"decoder_layers.{j}.up_sample_conv")
        self._pk_conv(pk, "decoder_conv_out", opad=8)
        pk.finalize()
        self.pack = pk

    # ------------------------------------------------------------------------------------------
    def forward(self, x, need_backward=True):
        """x: (B, im_channels, H, W) fp32 image. Returns (reconstruction NHWC fp32 [B*H*W, 8] with the first
        im_channels valid, ctx); ctx["vq_loss"] (1,) = mean((q - x)^2) (the codebook and the commitment loss share
        this value), ctx["indices"] (B, h, w) int64."""
        L, P = self.L, self.P
        B, Cx, H, W = x.shape
        assert Cx == self.im_channels
        G = L["G"]
        K.PHASE = "fwd"
        tape = Tape()
        st = dict(B=B, H=H, W=W)
        grads = Grads(self.device)
        x = plan.as_operand(x)
        d, m = L["down"], L["mid"]
        # ---- encoder (vqvae.py:128-137) ----
        tape.label = "encoder_in"
        xin = self._new(B * H * W, self.cin_pad)
        _lib.check(_lib.lib().sdmi_prep_input(x.data_ptr(), B, Cx, H, W, None, 0, 1, 1, None, 0, xin.data_ptr(),
                                              self.cin_pad, None, K._stream()), "sdmi_prep_input")
        cur, name = self._new(B * H * W, d[0]), "enc_in"
        K.conv_fwd(xin, B, H, W, self.cin_pad, self.cin_pad, self.W("encoder_conv_in#f"), d[0], 3, 3, 1, 1, cur, d[0],
                   bias=P["encoder_conv_in.bias"])
        grads.declare(name, B * H * W, d[0])
        tape.append((self._bwd_enc_in, dict(xin=xin, B=B, H=H, W=W)))
        h, w = H, W
        for i in range(len(d) - 1):
            p = f"encoder_layers.{i}"
            tape.label = p
            for l in range(L["n_down"]):
                cin = d[i] if l == 0 else d[i + 1]
                cur, name = self._op("res", p, l, cin, d[i + 1], cur, name, None, f"{p}.res{l}", B, h, w, st, tape,
                                     grads)
                if L["attn"][i]:
                    cur, name = self._op("self", p, l, d[i + 1], d[i + 1], cur, name, None, f"{p}.self{l}", B, h, w,
                                         st, tape, grads)
            if L["ds"][i]:
                cur, name = self._op("down", p, 0, d[i + 1], d[i + 1], cur, name, None, f"{p}.down", B, h, w, st,
                                     tape, grads)
                h, w = h // 2, w // 2
        for i in range(len(m) - 1):
            p = f"encoder_mids.{i}"
            tape.label = p
            cur, name = self._mid(p, cur, name, B, h, w, m[i], m[i + 1], st, tape, grads)
        tape.label = "encoder_out"
        Pn = h * w
        hs = self._new(B * Pn, d[-1])
        tab = K.gn_fwd(cur, B, Pn, d[-1], G, P["encoder_norm_out.weight"], P["encoder_norm_out.bias"], True, hs)
        z = self._new(B * Pn, 8, torch.float32)
        K.conv_fwd(hs, B, h, w, d[-1], d[-1], self.W("encoder_conv_out#f"), 8, 3, 3, 1, 1, z, 8,
                   bias=P["encoder_conv_out.bias"], n_store=L["z"])
        q = dict(B=B, h=h, w=w)  # state shared by the quantiser's backward entries
        tape.append((self._bwd_enc_out, dict(x=cur, xn=name, tab=tab, hs=hs, B=B, h=h, w=w, q=q)))
        # ---- quantiser (vqvae.py:93-126) ----
        zc = L["z"]
        zq = torch.empty(B, zc, h, w, dtype=torch.float32, device=self.device)
        pre = torch.empty_like(zq)
        idx = torch.empty(B, h, w, dtype=torch.int64, device=self.device)
        vq_loss = torch.empty(1, dtype=torch.float32, device=self.device)
        ws = torch.empty(_lib.lib().sdmi_vq_workspace(B * Pn) // 4 + 1, dtype=torch.float32, device=self.device)
        _lib.check(_lib.lib().sdmi_vq_quantize(z.data_ptr(), 8, P["pre_quant_conv.weight"].data_ptr(),
                                               P["pre_quant_conv.bias"].data_ptr(), P["embedding.weight"].data_ptr(),
                                               L["K"], B, Pn, zc, zq.data_ptr(), idx.data_ptr(), pre.data_ptr(),
                                               ws.data_ptr(), vq_loss.data_ptr(), K._stream()), "sdmi_vq_quantize")
        q.update(z=z, zq=zq, pre=pre, idx=idx)
        tape.label = "quant"
        tape.append((self._bwd_quant, dict(q=q)))
        # ---- decoder (vqvae.py:141-153) ----
        tape.label = "decoder_in"
        zin = self._new(B * Pn, 8)
        _lib.check(_lib.lib().sdmi_pointwise_in(zq.data_ptr(), B, zc, Pn, P["post_quant_conv.weight"].data_ptr(),
                                                P["post_quant_conv.bias"].data_ptr(), zc, zin.data_ptr(), 8,
                                                K._stream()), "sdmi_pointwise_in")
        cur, name = self._new(B * Pn, m[-1]), "dec_in"
        K.conv_fwd(zin, B, h, w, 8, 8, self.W("decoder_conv_in#f"), m[-1], 3, 3, 1, 1, cur, m[-1],
                   bias=P["decoder_conv_in.bias"])
        grads.declare(name, B * Pn, m[-1])
        tape.append((self._bwd_dec_in, dict(zin=zin, B=B, h=h, w=w, q=q)))
        for j, i in enumerate(reversed(range(1, len(m)))):
            p = f"decoder_mids.{j}"
            tape.label = p
            cur, name = self._mid(p, cur, name, B, h, w, m[i], m[i - 1], st, tape, grads)
        for j, i in enumerate(reversed(range(1, len(d)))):
            p = f"decoder_layers.{j}"
            tape.label = p
            if L["ds"][i - 1]:
                y = self._new(B * 4 * h * w, d[i])
                cur, name = self._op("up", p, 0, d[i], d[i], cur, name, y, f"{p}.up", B, h, w, st, tape, grads)
                h, w = 2 * h, 2 * w
            for l in range(L["n_up"]):
                cin = d[i] if l == 0 else d[i - 1]
                cur, name = self._op("res", p, l, cin, d[i - 1], cur, name, None, f"{p}.res{l}", B, h, w, st, tape,
                                     grads)
                if L["attn"][i - 1]:
                    cur, name = self._op("self", p, l, d[i - 1], d[i - 1], cur, name, None, f"{p}.self{l}", B, h, w,
                                         st, tape, grads)
        tape.label = "decoder_out"
        Pn = h * w
        hs = self._new(B * Pn, d[0])
        tab = K.gn_fwd(cur, B, Pn, d[0], G, P["decoder_norm_out.weight"], P["decoder_norm_out.bias"], True, hs)
        out = self._new(B * Pn, 8, torch.float32)
        K.conv_fwd(hs, B, h, w, d[0], d[0], self.W("decoder_conv_out#f"), 8, 3, 3, 1, 1, out, 8,
                   bias=P["decoder_conv_out.bias"], n_store=self.im_channels)
        tape.append((self._bwd_dec_out, dict(x=cur, xn=name, tab=tab, hs=hs, B=B, H=h, W=w)))
        ctx = dict(tape=tape, st=st, grads=grads, vq_loss=vq_loss, indices=idx, zq=zq, pre_quant=pre)
        if not need_backward:
            ctx.pop("tape")
        return out, ctx

    def _mid(self, p, cur, name, B, h, w, cin, cout, st, tape, grads):
        """MidBlock (blocks.py:225-267 at t_emb_dim=None): resnet, then [self-attention, resnet] x num_layers."""
        cur, name = self._op("res", p, 0, cin, cout, cur, name, None, f"{p}.res0", B, h, w, st, tape, grads)
        for l in range(self.L["n_mid"]):
            cur, name = self._op("self", p, l, cout, cout, cur, name, None, f"{p}.self{l}", B, h, w, st, tape, grads)
            cur, name = self._op("res", p, l + 1, cout, cout, cur, name, None, f"{p}.res{l + 1}", B, h, w, st, tape,
                                 grads)
        return cur, name

    # ---- backward of the head / latent interface ---------------------------------------------------------
    def _bwd_dec_out(self, c, grads):
        P, G = self.P, self.L["G"]
        B, H, W = c["B"], c["H"], c["W"]
        C = self.L["down"][0]
        Pn = H * W
        dout = self.dpred
        with self._wg(dout):
            K.conv_wgrad(dout, 8, c["hs"], B, H, W, C, C, 8, 3, 3, 1, 1, self.g("decoder_conv_out.weight"), H, W,
                         m_store=self.im_channels, bias_grad=self.g("decoder_conv_out.bias"))
        dhs = self._new(B * Pn, C)
        K.conv_fwd(dout, B, H, W, 8, 8, self.W("decoder_conv_out#d"), C, 3, 3, 1, 1, dhs, C)
        dx, fresh = grads.get(c["xn"])
        K.gn_bwd(c["x"], dhs, dx, c["tab"], P["decoder_norm_out.weight"], B, Pn, C, G, True,
                 self.g("decoder_norm_out.weight"), self.g("decoder_norm_out.bias"), addend=None if fresh else dx)

    def _bwd_dec_in(self, c, grads):
        """decoder_conv_in: weight gradient, and the data gradient into post_quant_conv's output (8-channel
        NHWC bf16, the z channels valid)."""
        B, h, w, q = c["B"], c["h"], c["w"], c["q"]
        m = self.L["mid"]
        dy, _ = grads.get("dec_in")
        ldy = K.ld_of(dy)
        with self._wg(dy):
            K.conv_wgrad(dy, ldy, c["zin"], B, h, w, 8, 8, m[-1], 3, 3, 1, 1, self.g("decoder_conv_in.weight"), h, w,
                         cvalid=self.L["z"], bias_grad=self.g("decoder_conv_in.bias"))
        dzin = self._new(B * h * w, 8)
        K.conv_fwd(dy, B, h, w, m[-1], ldy, self.W("decoder_conv_in#d"), 8, 3, 3, 1, 1, dzin, 8)
        q["dzin"] = dzin

    def _bwd_quant(self, c, grads):
        """sdmi_vq_bwd: post_quant_conv dW/db, straight-through + commitment gradient, pre_quant_conv dW/db, the
        codebook gradient and the gradient of encoder_conv_out's output (all on the critical path)."""
        q = c["q"]
        B, h, w = q["B"], q["h"], q["w"]
        L, P = self.L, self.P
        q["dz"] = dz = self._new(B * h * w, 8)
        ws = torch.empty(_lib.lib().sdmi_vq_bwd_workspace() // 4, dtype=torch.float32, device=self.device)
        _lib.check(_lib.lib().sdmi_vq_bwd(
            q["dzin"].data_ptr(), 8, q["zq"].data_ptr(), P["post_quant_conv.weight"].data_ptr(), q["pre"].data_ptr(),
            q["idx"].data_ptr(), P["embedding.weight"].data_ptr(), L["K"], q["z"].data_ptr(), 8,
            P["pre_quant_conv.weight"].data_ptr(), B, h * w, L["z"], self.commitment_beta, self.codebook_weight,
            dz.data_ptr(), 8, ws.data_ptr(), self.g("post_quant_conv.weight").data_ptr(),
            self.g("post_quant_conv.bias").data_ptr(), self.g("pre_quant_conv.weight").data_ptr(),
            self.g("pre_quant_conv.bias").data_ptr(), self.g("embedding.weight").data_ptr(), K._p(self.dzq_add),
            K._p(self.loss_w), K._stream()), "sdmi_vq_bwd")

    def _bwd_enc_out(self, c, grads):
        P, G = self.P, self.L["G"]
        B, h, w, q = c["B"], c["h"], c["w"], c["q"]
        C = self.L["down"][-1]
        Pn = h * w
        dz = q["dz"]
        with self._wg(dz):
            K.conv_wgrad(dz, 8, c["hs"], B, h, w, C, C, 8, 3, 3, 1, 1, self.g("encoder_conv_out.weight"), h, w,
                         m_store=self.L["z"], bias_grad=self.g("encoder_conv_out.bias"))
        dhs = self._new(B * Pn, C)
        K.conv_fwd(dz, B, h, w, 8, 8, self.W("encoder_conv_out#d"), C, 3, 3, 1, 1, dhs, C)
        dx, fresh = grads.get(c["xn"])
        K.gn_bwd(c["x"], dhs, dx, c["tab"], P["encoder_norm_out.weight"], B, Pn, C, G, True,
                 self.g("encoder_norm_out.weight"), self.g("encoder_norm_out.bias"), addend=None if fresh else dx)

    def _bwd_enc_in(self, c, grads):
        B, H, W = c["B"], c["H"], c["W"]
        C0 = self.L["down"][0]
        dy, _ = grads.get("enc_in")
        ldy = K.ld_of(dy)
        with self._wg(dy):
            K.conv_wgrad(dy, ldy, c["xin"], B, H, W, self.cin_pad, self.cin_pad, C0, 3, 3, 1, 1,
                         self.g("encoder_conv_in.weight"), H, W, cvalid=self.im_channels,
                         bias_grad=self.g("encoder_conv_in.bias"))

    # ------------------------------------------------------------------------------------------
    def backward(self, ctx, dout, codebook_weight=1.0, commitment_beta=0.2, grads=None, on_progress=None,
                 dzq=None, loss_w=None):
        """dout: NHWC bf16 [B*H*W, 8] = dL/d(reconstruction). The codebook / commitment terms enter at the
        quantiser with their weights (times the device scalars loss_w = {d codebook, d commitment} when given);
        dzq (NCHW fp32, optional): a gradient of the quantised latent from outside the decoder. Every parameter
        gradient is fully overwritten."""
        self.codebook_weight = float(codebook_weight)
        self.commitment_beta = float(commitment_beta)
        self.dzq_add, self.loss_w = dzq, loss_w
        if grads is not None:
            self.Gd = grads
        assert self.Gd is not None, "engine built without gradient buffers"
        self.dpred = dout
        tape, grads = ctx["tape"], ctx["grads"]
        K.PHASE = "bwd"
        for k in range(len(tape) - 1, -1, -1):
            fn, c = tape[k]
            fn(c, grads)
            if on_progress is not None:
                on_progress(tape, k)
        self._join()
        self._keep = []
        self.dpred = None
        K.PHASE = ""


class VQVAETrainer:
    """The generator step of train_vqvae_celebhq.py:405-470 without LPIPS / GAN: forward, recon MSE + codebook
    (weight codebook_weight) + commitment (commitment_beta) losses, backward, Adam(lr, betas=(0.5, 0.999)).
    Flat fp32 parameter / gradient / moment buffers; the step never synchronises with the host. With N > 1 ranks
    the gradients are averaged over the process group (one bucketed all-reduce after the backward) before Adam."""

    def __init__(self, cfg, state_dict, device, *, im_channels=3, lr=2e-5, betas=(0.5, 0.999), eps=1e-8,
                 codebook_weight=1.0, commitment_beta=0.2, group=None, bucket_bytes=64 << 20):
        from .reducer import BucketReducer
        self.cfg = cfg
        self.device = torch.device(device)
        shapes = {k: tuple(v.shape) for k, v in state_dict.items()}
        # flat order: the state-dict order reversed, so the backward finalises gradients roughly front to back
        self.store = FlatStore(shapes, cfg, self.device, order=list(reversed(list(shapes))))
        self.store.load(state_dict)
        self.group = group
        self.world = dist.get_world_size(group) if (group is not None or dist.is_initialized()) else 1
        if self.world > 1:
            src = 0 if group is None or group is dist.group.WORLD else dist.get_global_rank(group, 0)
            dist.broadcast(self.store.params, src=src, group=group)
        self.m = torch.zeros_like(self.store.params)
        self.v = torch.zeros_like(self.store.params)
        # optimizer state vector (csrc/optim.hip); loss scale 1 and no growth: the reference step is plain fp32
        self.state = torch.tensor([0, 0, 1.0, 0, 0, 0, 0, 0], dtype=torch.float32, device=self.device)
        self.hp = dict(lr=lr, b1=betas[0], b2=betas[1], eps=eps, cw=codebook_weight, beta=commitment_beta)
        self.engine = VQVAETrainEngine(cfg, self.store.p, self.store.g, im_channels=im_channels)
        self.reducer = BucketReducer(self.store.grads, group, bucket_bytes) if self.world > 1 else None
        if self.reducer is not None and self.engine.side is not None:
            self.reducer.producers.append(self.engine.side)
        self.engine.refresh_weights()
        self.vq_loss = None
        self.indices = None

    def step(self, im):
        """One generator step on a device image batch (B, im_channels, H, W) fp32 in [-1, 1]."""
        eng, st, hp = self.engine, self.store, self.hp
        B, C, H, W = im.shape
        self._shape = (B, C, H, W)
        out, ctx = eng.forward(im)
        dout = eng.new_dpred(B, H, W)
        K.mse(out, 8, plan.as_operand(im), B, C, H * W, 1.0, dout, self.state[S_LOSS:S_LOSS + 1])
        if self.reducer is not None:
            self.reducer.reset()
        eng.backward(ctx, dout, hp["cw"], hp["beta"])
        if self.reducer is not None:
            self.reducer.ready(st.numel)
            self.reducer.finish()
        self.vq_loss, self.indices, self.out = ctx["vq_loss"], ctx["indices"], out
        L = _lib.lib()
        wsb = L.sdmi_optim_workspace_for(st.numel)
        ws = torch.empty(wsb // 4, dtype=torch.float32, device=self.device)
        # no loss scaler (growth_interval 0: the scale stays 1) and no clipping (max norm inf): the gradient
        # coefficient is exactly 1 / world. A non-finite gradient skips the update instead of poisoning the weights.
        _lib.check(L.sdmi_clip_unscale_ws(st.grads.data_ptr(), st.numel, float("inf"), self.state.data_ptr(),
                                          ws.data_ptr(), wsb, 0, 0, float(self.world), K._stream()),
                   "sdmi_clip_unscale_ws")
        _lib.check(L.sdmi_adam_ema(st.params.data_ptr(), st.grads.data_ptr(), self.m.data_ptr(), self.v.data_ptr(),
                                   None, st.numel, self.state.data_ptr(), hp["lr"], hp["b1"], hp["b2"], hp["eps"], 0.0,
                                   1.0, K._stream()), "sdmi_adam_ema")
        eng.refresh_weights()
        return self.state

    def losses(self):
        """Host dict of the last step's losses (synchronises): recon, codebook (weighted), commitment (weighted)."""
        rec = self.state[S_LOSS].item()
        vq = self.vq_loss.item()
        return dict(recon=rec, codebook=self.hp["cw"] * vq, commitment=self.hp["beta"] * vq,
                    total=rec + (self.hp["cw"] + self.hp["beta"]) * vq)

    def reconstruction(self):
        """The last step's decoder output as (B, im_channels, H, W) fp32."""
        B, C, H, W = self._shape
        return self.engine.pred_to_nchw(self.out, B, H, W)

    def state_dict(self):
        return {k: self.store.p[k] for k in self.store.shapes}
