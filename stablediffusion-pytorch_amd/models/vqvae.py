"""Drop-in VQVAE (reference models/vqvae.py:6-158) on the MI355X HIP path.

Same constructor, assertions, module tree and state-dict keys as the reference (encoder_conv_in,
encoder_layers / encoder_mids (DownBlock / MidBlock), encoder_norm_out, encoder_conv_out, pre_quant_conv,
embedding, post_quant_conv, decoder_conv_in, decoder_mids, decoder_layers (UpBlock), decoder_norm_out,
decoder_conv_out), so gen_vqvae_latents.py / sample_ddpm_*.py load a reference checkpoint and call
`encode(im)` -> (z, {'codebook_loss', 'commitment_loss'}), `decode(z)` and `forward(x)` -> (out, z, losses)
unchanged. encode / decode run as one schedule of gfx950 kernels (sdmi.vqvae_engine) in inference mode
(the reference's latent-generation and decoding path). forward(x) with autograd enabled runs the training
engine (sdmi.vqvae_train) as one autograd Function: train_vqvae_celebhq.py:414-441 then computes its losses on
the returned (out, z, {'codebook_loss', 'commitment_loss'}) and calls .backward() unchanged -- the gradients of
the reconstruction (MSE, LPIPS, GAN terms: any torch loss), of z and of both quantiser losses flow back through
the straight-through estimator into every parameter.
"""
import torch
import torch.nn as nn

from models.blocks import DownBlock, MidBlock, UpBlock
from sdmi import _lib
from sdmi import leaf as LF
from sdmi.vqvae_engine import VQVAEEngine
from sdmi.vqvae_train import VQVAETrainEngine


class VQVAEFunction(torch.autograd.Function):
    """(x, *params) -> (reconstruction, z_q, codebook_loss, commitment_loss) on the HIP training engine."""

    @staticmethod
    def forward(ctx, mod, x, *params):
        eng = mod._train_eng(x)
        B, C, H, W = x.shape
        out, c = eng.forward(x)
        ctx.mod, ctx.c, ctx.hw = mod, c, (B, H, W)
        vq = c["vq_loss"].reshape(())
        return eng.pred_to_nchw(out, B, H, W), c["zq"], vq.clone(), vq.clone()

    @staticmethod
    def backward(ctx, dimg, dz, dcb, dcm):
        mod = ctx.mod
        eng = mod._tengine
        B, H, W = ctx.hw
        dev = eng.device
        dout = (eng.dpred_from_nchw(dimg.float().contiguous()) if dimg is not None
                else torch.zeros(B * H * W, 8, dtype=torch.bfloat16, device=dev))
        zero = torch.zeros((), device=dev)
        loss_w = torch.stack([(dcb if dcb is not None else zero).float().reshape(()),
                              (dcm if dcm is not None else zero).float().reshape(())])
        names = [k for k, _ in mod.named_parameters()]
        params = dict(mod.named_parameters())
        grads = {k: torch.empty_like(params[k]) for k in names}
        eng.backward(ctx.c, dout, 1.0, 1.0, grads=grads, dzq=dz.float().contiguous() if dz is not None else None,
                     loss_w=loss_w)
        ctx.c = None
        return (None, None) + tuple(grads[k] for k in names)


class VQVAE(nn.Module):
    def __init__(self, im_channels, model_config):
        super().__init__()
        cfg = model_config
        self.im_channels = im_channels
        self.down_channels = cfg["down_channels"]
        self.mid_channels = cfg["mid_channels"]
        self.down_sample = cfg["down_sample"]
        self.num_down_layers = cfg["num_down_layers"]
        self.num_mid_layers = cfg["num_mid_layers"]
        self.num_up_layers = cfg["num_up_layers"]
        self.attns = cfg["attn_down"]
        self.z_channels = cfg["z_channels"]
        self.codebook_size = cfg["codebook_size"]
        self.norm_channels = cfg["norm_channels"]
        self.num_heads = cfg["num_heads"]
        assert self.mid_channels[0] == self.down_channels[-1]
        assert self.mid_channels[-1] == self.down_channels[-1]
        assert len(self.down_sample) == len(self.down_channels) - 1
        assert len(self.attns) == len(self.down_channels) - 1
        self.up_sample = list(reversed(self.down_sample))
        dc, mc = self.down_channels, self.mid_channels
        self.encoder_conv_in = nn.Conv2d(im_channels, dc[0], kernel_size=3, padding=(1, 1))
        self.encoder_layers = nn.ModuleList([
            DownBlock(dc[i], dc[i + 1], t_emb_dim=None, down_sample=self.down_sample[i], num_heads=self.num_heads,
                      num_layers=self.num_down_layers, attn=self.attns[i], norm_channels=self.norm_channels)
            for i in range(len(dc) - 1)])
        self.encoder_mids = nn.ModuleList([
            MidBlock(mc[i], mc[i + 1], t_emb_dim=None, num_heads=self.num_heads, num_layers=self.num_mid_layers,
                     norm_channels=self.norm_channels)
            for i in range(len(mc) - 1)])
        self.encoder_norm_out = nn.GroupNorm(self.norm_channels, dc[-1])
        self.encoder_conv_out = nn.Conv2d(dc[-1], self.z_channels, kernel_size=3, padding=1)
        self.pre_quant_conv = nn.Conv2d(self.z_channels, self.z_channels, kernel_size=1)
        self.embedding = nn.Embedding(self.codebook_size, self.z_channels)
        self.post_quant_conv = nn.Conv2d(self.z_channels, self.z_channels, kernel_size=1)
        self.decoder_conv_in = nn.Conv2d(self.z_channels, mc[-1], kernel_size=3, padding=(1, 1))
        self.decoder_mids = nn.ModuleList([
            MidBlock(mc[i], mc[i - 1], t_emb_dim=None, num_heads=self.num_heads, num_layers=self.num_mid_layers,
                     norm_channels=self.norm_channels)
            for i in reversed(range(1, len(mc)))])
        self.decoder_layers = nn.ModuleList([
            UpBlock(dc[i], dc[i - 1], t_emb_dim=None, up_sample=self.down_sample[i - 1], num_heads=self.num_heads,
                    num_layers=self.num_up_layers, attn=self.attns[i - 1], norm_channels=self.norm_channels)
            for i in reversed(range(1, len(dc)))])
        self.decoder_norm_out = nn.GroupNorm(self.norm_channels, dc[0])
        self.decoder_conv_out = nn.Conv2d(dc[0], im_channels, kernel_size=3, padding=1)
        self._engine = None
        self._ptrs = None

    def _eng(self, t):
        if not t.is_cuda:
            raise RuntimeError("the sdmi VQVAE runs on the MI355X HIP path only (move the model and inputs to cuda)")
        _lib.lib()
        params = dict(self.named_parameters())
        ptrs = [p.data_ptr() for p in params.values()]
        if self._engine is None or ptrs != self._ptrs:
            self._engine = VQVAEEngine(self.model_config_dict(), {k: v.detach() for k, v in params.items()},
                                       im_channels=self.im_channels)
            self._ptrs = ptrs
        self._engine.refresh_weights()  # bf16 GEMM-layout copies of the (possibly updated) fp32 weights
        return self._engine

    def _train_eng(self, t):
        if not t.is_cuda:
            raise RuntimeError("the sdmi VQVAE runs on the MI355X HIP path only (move the model and inputs to cuda)")
        _lib.lib()
        params = dict(self.named_parameters())
        ptrs = [p.data_ptr() for p in params.values()]
        if getattr(self, "_tengine", None) is None or ptrs != self._tptrs:
            self._tengine = VQVAETrainEngine(self.model_config_dict(), {k: v.detach() for k, v in params.items()},
                                             im_channels=self.im_channels)
            self._tptrs = ptrs
            self._tsig = None
        sig = tuple(p._version for p in params.values())
        # grad-enabled (training) calls repack every time: `.data` writes keep the version counter
        if torch.is_grad_enabled() or sig != self._tsig:
            self._tengine.refresh_weights()
            self._tsig = sig
        return self._tengine

    def model_config_dict(self):
        return {"down_channels": self.down_channels, "mid_channels": self.mid_channels,
                "down_sample": self.down_sample, "attn_down": self.attns, "num_down_layers": self.num_down_layers,
                "num_mid_layers": self.num_mid_layers, "num_up_layers": self.num_up_layers,
                "z_channels": self.z_channels, "codebook_size": self.codebook_size,
                "norm_channels": self.norm_channels, "num_heads": self.num_heads}

    def _leaf(self):
        """Leaf-by-leaf path (sdmi.leaf): a swapped leaf or sdmi_leaf_path = True."""
        return getattr(self, "sdmi_leaf_path", False) or not LF.engine_ok(self, (VQVAE, DownBlock, MidBlock, UpBlock))

    def quantize(self, x):
        """vqvae.py:93-126 on its own (pre-quantisation latent -> z_q, losses, indices)."""
        return LF.quantize(self.embedding, x)

    def _leaf_encode(self, x):
        out = LF.call(self.encoder_conv_in, x)
        for down in self.encoder_layers:
            out = down(out)
        for mid in self.encoder_mids:
            out = mid(out)
        out = LF.call(nn.Sequential(self.encoder_norm_out, nn.SiLU()), out)
        out = LF.call(self.pre_quant_conv, LF.call(self.encoder_conv_out, out))
        return self.quantize(out)

    def _leaf_decode(self, z):
        out = LF.call(self.decoder_conv_in, LF.call(self.post_quant_conv, z))
        for mid in self.decoder_mids:
            out = mid(out)
        for up in self.decoder_layers:
            out = up(out)
        out = LF.call(nn.Sequential(self.decoder_norm_out, nn.SiLU()), out)
        return LF.call(self.decoder_conv_out, out)

    @torch.no_grad()
    def quantize_indices(self, x):
        """Encode and also return the codebook indices (B, h, w) int64 (vqvae.py:124-125)."""
        if self._leaf():
            zq, losses, idx = self._leaf_encode(x)
            return zq, losses["codebook_loss"].reshape(1), idx
        return self._eng(x).encode(x)

    def encode(self, x):
        if self._leaf():
            zq, losses, _ = self._leaf_encode(x)
            return zq, losses
        with torch.no_grad():
            zq, loss, _ = self._eng(x).encode(x)
        return zq, {"codebook_loss": loss[0], "commitment_loss": loss[0]}

    def decode(self, z):
        if self._leaf():
            return self._leaf_decode(z)
        with torch.no_grad():
            return self._eng(z).decode(z)

    def forward(self, x):
        if self._leaf():
            z, losses, _ = self._leaf_encode(x)
            return self._leaf_decode(z), z, losses
        if torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters()):
            out, z, cb, cm = VQVAEFunction.apply(self, x, *self.parameters())
            return out, z, {"codebook_loss": cb, "commitment_loss": cm}
        z, quant_losses = self.encode(x)
        return self.decode(z), z, quant_losses
