"""VQVAE encode / quantize / decode (reference models/vqvae.py:93-153 with models/blocks.py DownBlock :27-146,
MidBlock :149-267, UpBlock :270-370 at t_emb_dim=None) as one schedule of gfx950 kernels.

MI355X plan: activations are NHWC bf16 [pixels, C]; every 3x3 conv is one implicit-GEMM launch with the
resnet's second conv and 1x1 residual conv fused into ONE GEMM by K-concatenation; the stride-2 4x4 convs are
one strided implicit GEMM, the transposed convs four sub-pixel GEMMs; GroupNorm(+SiLU) are the strip
reduction + apply kernels; the mid-block self-attention is the fused flash kernel (heads 4 x 64); the
encoder head writes fp32 and the pre_quant_conv + nearest-codebook search + straight-through output run
in one kernel (sdmi_vq_quantize), so the latent never round-trips through bf16. Forward only (the
reference's latent generation / decoding path, gen_vqvae_latents.py:89-106, sample_ddpm_*.py)."""
import torch

from . import _lib
from . import kernels as K
from . import plan
from .unet_engine import PackPlan


def vqvae_layout(cfg):
    return dict(down=list(cfg["down_channels"]), mid=list(cfg["mid_channels"]), ds=list(cfg["down_sample"]),
                attn=list(cfg["attn_down"]), n_down=cfg["num_down_layers"], n_mid=cfg["num_mid_layers"],
                n_up=cfg["num_up_layers"], z=cfg["z_channels"], K=cfg["codebook_size"], G=cfg["norm_channels"],
                heads=cfg["num_heads"])


class VQVAEEngine:
    def __init__(self, cfg, params, im_channels=3):
        self.cfg = cfg
        self.L = vqvae_layout(cfg)
        L = self.L
        if L["z"] > 8:
            raise ValueError("z_channels > 8 is not supported by sdmi_vq_quantize")
        for c in L["down"] + L["mid"]:
            if c % 8:
                raise ValueError("channel counts must be multiples of 8")
        self.P = params
        self.im_channels = im_channels
        self.device = next(iter(params.values())).device
        self.cin_pad = (im_channels + 7) // 8 * 8
        self._build_pack()

    # ------------------------------------------------------------------------------------------
    def _resnets(self):
        """(prefix, index, cin, cout) of every resnet (encoder and decoder)."""
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
        P, L = self.P, self.L
        pk = PackPlan(self.device)

        def conv(key, ipad=None, opad=None):
            w = P[key + ".weight"]
            O, I, KH, KW = w.shape
            pk.add(key, w, O, I, ipad or I, KH, KW, I * KH * KW, KH * KW, KW, 1, rows=opad)

        def lin(key, name):
            w = P[key]
            N, Kd = w.shape
            pk.add(name, w, N, Kd, Kd, 1, 1, Kd, 1, 0, 0)

        conv("encoder_conv_in", ipad=self.cin_pad)
        for (p, l, cin, cout) in self._resnets():
            conv(f"{p}.resnet_conv_first.{l}.2")
            w2 = P[f"{p}.resnet_conv_second.{l}.2.weight"]
            wr = P[f"{p}.residual_input_conv.{l}.weight"]
            cat = f"{p}.res{l}#cat"  # [cout][9*cout + cin]: second conv | 1x1 residual conv
            pk.reserve(cat, cout, 9 * cout + cin)
            pk.add(None, w2, cout, cout, cout, 3, 3, cout * 9, 9, 3, 1, into=cat)
            pk.add(None, wr, cout, cin, cin, 1, 1, cin, 1, 0, 0, into=cat, col0=9 * cout)
        for key in self._attn_keys():
            lin(key + ".in_proj_weight", key + "#in")
            lin(key + ".out_proj.weight", key + "#out")
        d = L["down"]
        for i in range(len(d) - 1):
            if L["ds"][i]:
                conv(f"encoder_layers.{i}.down_sample_conv")
        conv("encoder_conv_out", opad=8)
        conv("decoder_conv_in", ipad=8)
        for j, i in enumerate(reversed(range(1, len(d)))):
            if L["ds"][i - 1]:
                key = f"decoder_layers.{j}.up_sample_conv"
                w = P[key + ".weight"]  # ConvTranspose2d (Cx, Cy, 4, 4)
                Cx, Cy = w.shape[0], w.shape[1]
                for ph in range(2):
                    for pw in range(2):  # sub-pixel phase weights [co][a][b][ci] = W[ci][co][3-ph-2a][3-pw-2b]
                        pk.add(f"{key}#f{ph}{pw}", w, Cy, Cx, Cx, 2, 2, 16, Cy * 16, 4, 1, 3 - ph, -2, 3 - pw, -2)
        conv("decoder_conv_out", opad=8)
        pk.finalize()
        self.pack = pk

    def W(self, name):
        return self.pack.view(name)

    def refresh_weights(self):
        if self.pack.stale():
            self.pack.finalize()
        self.pack.run()

    def _new(self, rows, C, dtype=torch.bfloat16):
        return torch.empty(rows, C, dtype=dtype, device=self.device)

    # ------------------------------------------------------------------------------------------
    def _resnet(self, p, l, cin, cout, x, B, h, w):
        P, G = self.P, self.L["G"]
        Pn = h * w
        a, b = f"{p}.resnet_conv_first.{l}", f"{p}.resnet_conv_second.{l}"
        h0 = self._new(B * Pn, cin)
        t1 = K.gn_fwd(x, B, Pn, cin, G, P[a + ".0.weight"], P[a + ".0.bias"], True, h0)
        h1 = self._new(B * Pn, cout)
        K.conv_fwd(h0, B, h, w, cin, cin, self.W(a + ".2"), cout, 3, 3, 1, 1, h1, cout, bias=P[a + ".2.bias"])
        del h0
        h2 = self._new(B * Pn, cout)
        t2 = K.gn_fwd(h1, B, Pn, cout, G, P[b + ".0.weight"], P[b + ".0.bias"], True, h2)
        del h1
        y = self._new(B * Pn, cout)
        K.conv_fwd(h2, B, h, w, cout, cout, self.W(f"{p}.res{l}#cat"), cout, 3, 3, 1, 1, y, cout,
                   bias=P[b + ".2.bias"], x2=x, cin2=cin, bias2=P[f"{p}.residual_input_conv.{l}.bias"])
        return y

    def _attn(self, p, l, C, x, B, h, w):
        P, G, Hh = self.P, self.L["G"], self.L["heads"]
        N = h * w
        nk, mk = f"{p}.attention_norms.{l}", f"{p}.attentions.{l}"
        a = self._new(B * N, C)
        tab = K.gn_fwd(x, B, N, C, G, P[nk + ".weight"], P[nk + ".bias"], False, a)
        qkv = self._new(B * N, 3 * C)
        K.linear(a, self.W(mk + "#in"), qkv, bias=P[mk + ".in_proj_bias"])
        o = self._new(B * N, C)
        K.attn_fwd(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], o, B, Hh, N, N, C // Hh)
        y = self._new(B * N, C)
        K.linear(o, self.W(mk + "#out"), y, bias=P[mk + ".out_proj.bias"], resid=x)
        return y

    def _mid(self, p, x, B, h, w, cin, cout):
        x = self._resnet(p, 0, cin, cout, x, B, h, w)
        for l in range(self.L["n_mid"]):
            x = self._attn(p, l, cout, x, B, h, w)
            x = self._resnet(p, l + 1, cout, cout, x, B, h, w)
        return x

    def _head(self, key_norm, key_conv, x, B, h, w, C, n_store):
        P = self.P
        hs = self._new(B * h * w, C)
        tab = K.gn_fwd(x, B, h * w, C, self.L["G"], P[key_norm + ".weight"], P[key_norm + ".bias"], True, hs)
        out = self._new(B * h * w, 8, torch.float32)
        K.conv_fwd(hs, B, h, w, C, C, self.W(key_conv), 8, 3, 3, 1, 1, out, 8, bias=P[key_conv + ".bias"],
                   n_store=n_store)
        return out

    # ------------------------------------------------------------------------------------------
    def encode(self, x, want_pre_quant=False):
        """vqvae.py:128-139. x: (B, 3, H, W) fp32 -> (z_q NCHW fp32, loss (1,), indices int64 (B, h, w)
        [, pre-quantisation latent NCHW fp32])."""
        L, P = self.L, self.P
        B, Cx, H, W = x.shape
        assert Cx == self.im_channels
        x = plan.as_operand(x)
        xin = self._new(B * H * W, self.cin_pad)
        _lib.check(_lib.lib().sdmi_prep_input(x.data_ptr(), B, Cx, H, W, None, 0, 1, 1, None, 0, xin.data_ptr(),
                                              self.cin_pad, None, K._stream()), "sdmi_prep_input")
        d = L["down"]
        cur = self._new(B * H * W, d[0])
        K.conv_fwd(xin, B, H, W, self.cin_pad, self.cin_pad, self.W("encoder_conv_in"), d[0], 3, 3, 1, 1, cur, d[0],
                   bias=P["encoder_conv_in.bias"])
        del xin
        h, w = H, W
        for i in range(len(d) - 1):
            p = f"encoder_layers.{i}"
            for l in range(L["n_down"]):
                cur = self._resnet(p, l, d[i] if l == 0 else d[i + 1], d[i + 1], cur, B, h, w)
                if L["attn"][i]:
                    cur = self._attn(p, l, d[i + 1], cur, B, h, w)
            if L["ds"][i]:
                y = self._new(B * (h // 2) * (w // 2), d[i + 1])
                K.conv_fwd(cur, B, h, w, d[i + 1], d[i + 1], self.W(f"{p}.down_sample_conv"), d[i + 1], 4, 4, 2, 1, y,
                           d[i + 1], bias=P[f"{p}.down_sample_conv.bias"])
                cur = y
                h, w = h // 2, w // 2
        m = L["mid"]
        for i in range(len(m) - 1):
            cur = self._mid(f"encoder_mids.{i}", cur, B, h, w, m[i], m[i + 1])
        z = self._head("encoder_norm_out", "encoder_conv_out", cur, B, h, w, d[-1], L["z"])
        zq = torch.empty(B, L["z"], h, w, dtype=torch.float32, device=self.device)
        idx = torch.empty(B, h, w, dtype=torch.int64, device=self.device)
        pre = torch.empty_like(zq) if want_pre_quant else None
        loss = torch.empty(1, dtype=torch.float32, device=self.device)
        ws = torch.empty(_lib.lib().sdmi_vq_workspace(B * h * w) // 4 + 1, dtype=torch.float32, device=self.device)
        _lib.check(_lib.lib().sdmi_vq_quantize(z.data_ptr(), 8, P["pre_quant_conv.weight"].data_ptr(),
                                               P["pre_quant_conv.bias"].data_ptr(), P["embedding.weight"].data_ptr(),
                                               L["K"], B, h * w, L["z"], zq.data_ptr(), idx.data_ptr(), K._p(pre),
                                               ws.data_ptr(), loss.data_ptr(), K._stream()), "sdmi_vq_quantize")
        if want_pre_quant:
            return zq, loss, idx, pre
        return zq, loss, idx

    def decode(self, z):
        """vqvae.py:141-153. z: (B, z_channels, h, w) fp32 -> (B, 3, h*2^n, w*2^n) fp32."""
        L, P = self.L, self.P
        B, Cz, h, w = z.shape
        assert Cz == L["z"]
        z = plan.as_operand(z)
        zin = self._new(B * h * w, 8)
        _lib.check(_lib.lib().sdmi_pointwise_in(z.data_ptr(), B, Cz, h * w, P["post_quant_conv.weight"].data_ptr(),
                                                P["post_quant_conv.bias"].data_ptr(), Cz, zin.data_ptr(), 8,
                                                K._stream()), "sdmi_pointwise_in")
        m, d = L["mid"], L["down"]
        cur = self._new(B * h * w, m[-1])
        K.conv_fwd(zin, B, h, w, 8, 8, self.W("decoder_conv_in"), m[-1], 3, 3, 1, 1, cur, m[-1],
                   bias=P["decoder_conv_in.bias"])
        for j, i in enumerate(reversed(range(1, len(m)))):
            cur = self._mid(f"decoder_mids.{j}", cur, B, h, w, m[i], m[i - 1])
        for j, i in enumerate(reversed(range(1, len(d)))):
            p = f"decoder_layers.{j}"
            if L["ds"][i - 1]:
                key = f"{p}.up_sample_conv"
                wph = [self.W(f"{key}#f{ph}{pw}") for ph in range(2) for pw in range(2)]
                y = self._new(B * 4 * h * w, d[i])
                K.convT_fwd_phases(cur, B, h, w, d[i], d[i], wph, d[i], y, d[i], bias=P[key + ".bias"])
                cur = y
                h, w = 2 * h, 2 * w
            for l in range(L["n_up"]):
                cur = self._resnet(p, l, d[i] if l == 0 else d[i - 1], d[i - 1], cur, B, h, w)
                if L["attn"][i - 1]:
                    cur = self._attn(p, l, d[i - 1], cur, B, h, w)
        out = self._head("decoder_norm_out", "decoder_conv_out", cur, B, h, w, d[0], self.im_channels)
        img = torch.empty(B, self.im_channels, h, w, dtype=torch.float32, device=self.device)
        _lib.check(_lib.lib().sdmi_nhwc_to_nchw(out.data_ptr(), 1, 8, B, self.im_channels, h * w, img.data_ptr(),
                                                K._stream()), "sdmi_nhwc_to_nchw")
        return img
