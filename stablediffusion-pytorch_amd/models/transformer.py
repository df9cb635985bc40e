"""Drop-in DiT (reference models/transformer.py:43-213) on the MI355X HIP path.

Same constructor, forward signature, assertions, initialisation and state-dict keys as the reference:
callers such as Model_DiT_12L_train.py:478-481 construct `DIT(im_channels, model_config)` and call
`model(x, t, cond_input)` unchanged. The whole forward and backward run as one explicit schedule of
gfx950 kernels (sdmi.dit_engine); parameters live in a flat fp32 store the first time the model runs on
the GPU. There is no CPU path: CPU inputs raise. With a swapped leaf or sdmi_leaf_path = True
the forward composes the layers like transformer.py:153-213, every leaf on the HIP per-op path (sdmi.leaf).
"""
import torch
import torch.nn as nn

from models.patch_embed import PatchEmbedding
from models.transformer_layer import TransformerLayer
from utils.config_utils import (get_config_value, validate_class_config, validate_class_conditional_input,
                                validate_image_config, validate_image_conditional_input, validate_text_config)
from sdmi import leaf as LF
from sdmi.module_glue import EngineHolder, invalidate_module, run_denoiser


def get_time_embedding(time_steps, temb_dim):
    """Sinusoidal embedding (transformer.py:18-40); host-side API mirror of sdmi_time_embedding."""
    assert temb_dim % 2 == 0, "time embedding dimension must be divisible by 2"
    half = temb_dim // 2
    factor = 10000 ** (torch.arange(0, half, dtype=torch.float32, device=time_steps.device) / half)
    arg = time_steps[:, None].repeat(1, half) / factor
    return torch.cat([torch.sin(arg), torch.cos(arg)], dim=-1)


class DIT(nn.Module):
    def __init__(self, im_channels, model_config, image_size=None):
        super().__init__()
        cfg = model_config
        self.image_height = image_size
        self.image_width = image_size
        self.im_channels = im_channels
        self.hidden_size = cfg["hidden_size"]
        self.patch_height = cfg["patch_size"]
        self.patch_width = cfg["patch_size"]
        self.timestep_emb_dim = cfg["timestep_emb_dim"]
        self.num_layers = cfg["num_layers"]
        self.num_heads = cfg["num_heads"]
        self.head_dim = cfg["head_dim"]
        self.class_cond = self.text_cond = self.image_cond = False
        self.text_embed_dim = None
        self.condition_config = get_config_value(cfg, "condition_config", None)
        if self.condition_config is not None:
            assert "condition_types" in self.condition_config, "Condition Type not provided in model config"
            types = self.condition_config["condition_types"]
            if "class" in types:
                validate_class_config(self.condition_config)
                self.class_cond = True
                self.num_classes = self.condition_config["class_condition_config"]["num_classes"]
            if "text" in types:
                validate_text_config(self.condition_config)
                self.text_cond = True
                self.text_embed_dim = self.condition_config["text_condition_config"]["text_embed_dim"]
            if "image" in types:
                validate_image_config(self.condition_config)
                self.image_cond = True
                ic = self.condition_config["image_condition_config"]
                self.im_cond_input_ch = ic["image_condition_input_channels"]
                self.im_cond_output_ch = ic["image_condition_output_channels"]
        if self.class_cond:
            self.class_emb = nn.Embedding(self.num_classes, self.timestep_emb_dim)
        if self.image_cond:
            self.cond_conv_in = nn.Conv2d(self.im_cond_input_ch, self.im_cond_output_ch, kernel_size=1, bias=False)
            patch_in = im_channels + self.im_cond_output_ch
        else:
            patch_in = im_channels
        self.cond = self.text_cond or self.image_cond or self.class_cond
        self.patch_embed_layer = PatchEmbedding(self.image_height or 0, self.image_width or 0, patch_in,
                                                self.patch_height, self.patch_width, self.hidden_size)
        self.t_proj = nn.Sequential(nn.Linear(self.timestep_emb_dim, self.hidden_size), nn.ReLU(),
                                    nn.Linear(self.hidden_size, self.hidden_size))
        layer_config = {"hidden_size": self.hidden_size, "num_heads": self.num_heads, "head_dim": self.head_dim}
        self.transformer_layers = nn.ModuleList([
            TransformerLayer(layer_config, cross_attn=self.text_cond,
                             context_dim=self.text_embed_dim if self.text_cond else None)
            for _ in range(self.num_layers)])
        self.norm = nn.LayerNorm(self.hidden_size, elementwise_affine=False, eps=1E-6)
        self.adaptive_norm_layer = nn.Sequential(nn.ReLU(), nn.Linear(self.hidden_size, 2 * self.hidden_size, bias=True))
        self.proj_out = nn.Linear(self.hidden_size, self.patch_height * self.patch_width * self.im_channels)
        nn.init.normal_(self.t_proj[0].weight, std=0.02)
        nn.init.normal_(self.t_proj[2].weight, std=0.02)
        nn.init.constant_(self.adaptive_norm_layer[-1].weight, 0)
        nn.init.constant_(self.adaptive_norm_layer[-1].bias, 0)
        nn.init.constant_(self.proj_out.weight, 0)
        nn.init.constant_(self.proj_out.bias, 0)
        self._sdmi = EngineHolder(self, cfg, "dit")

    def forward(self, x, t, cond_input=None):
        if self.cond:
            assert cond_input is not None, "Model initialized with conditioning so cond_input cannot be None"
        mask = text = klass = None
        if self.image_cond:
            validate_image_conditional_input(cond_input, x)
            mask = cond_input["image"]
        if self.class_cond:
            validate_class_conditional_input(cond_input, x, self.num_classes)
            klass = cond_input["class"]
        if self.text_cond:
            assert "text" in cond_input, \
                "Model initialized with text conditioning but cond_input has no text information"
            text = cond_input["text"]
        if getattr(self, "sdmi_leaf_path", False) or not self._sdmi_engine_ok():
            return self._leaf_forward(x, t, text, mask, klass)
        return run_denoiser(self, self._sdmi, x, t, text, mask, klass)

    def _sdmi_engine_ok(self):
        from models.attention import Attention
        from models.multihead_attention import CustomMultiheadAttention
        return LF.engine_ok(self, (DIT, PatchEmbedding, TransformerLayer, Attention, CustomMultiheadAttention))

    def sdmi_invalidate(self):
        """Repack the bf16 weights at the next forward (after writing parameters through `.data`)."""
        invalidate_module(self)

    def _leaf_forward(self, x, t, text, mask, klass):
        patch_source = x
        if self.image_cond:
            im_cond = LF.resize_nearest(mask.to(device=x.device, dtype=torch.float32), x.shape[-2:])
            patch_source = LF.cat_channels([patch_source, LF.call(self.cond_conv_in, im_cond)])
        out = self.patch_embed_layer(patch_source)
        t_emb = LF.time_embedding(t, x.shape[0], self.timestep_emb_dim, x.device)
        if self.class_cond:
            t_emb = t_emb + LF.class_embed(self.class_emb, klass)
        t_emb = LF.call(self.t_proj, t_emb)
        for layer in self.transformer_layers:
            out = layer(out, t_emb, text)
        shift, scale = LF.call(self.adaptive_norm_layer, t_emb).chunk(2, dim=1)
        out = LF.modulate(LF.call(self.norm, out), scale, shift)  # norm(out) * (1 + scale) + shift
        out = LF.call(self.proj_out, out)
        B, _, H, W = x.shape
        ph, pw = self.patch_height, self.patch_width
        nh, nw = H // ph, W // pw
        # 'b (nh nw) (ph pw c) -> b c (nh ph) (nw pw)'
        return out.reshape(B, nh, nw, ph, pw, self.im_channels).permute(0, 5, 1, 3, 2, 4).reshape(
            B, self.im_channels, H, W)
