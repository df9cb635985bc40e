"""Drop-in conditional UNet (reference models/unet_cond_base.py:9-183) on the MI355X HIP path.

Same constructor, forward signature, assertions and state-dict keys as the reference: callers such
as train_ddpm_cond_celebhq_multi_gpu.py:235-238 and tools/sample_ddpm_text_image_cond.py construct
`Unet(im_channels, model_config)` and call `model(x, t, cond_input)` unchanged. The forward and
backward run as one explicit schedule of gfx950 kernels (sdmi.unet_engine); parameters live in a
flat fp32 store the first time the model runs on the GPU. Once a leaf is no longer an exact torch type (a
swapped quantised layer) -- or with `sdmi_leaf_path = True` -- the forward composes the blocks
and leaves like the reference (unet_cond_base.py:124-183) on the per-op HIP path of sdmi.leaf instead.
"""
import torch
import torch.nn as nn

from models.blocks import DownBlock, MidBlock, UpBlockUnet, get_time_embedding  # noqa: F401
from utils.config_utils import (get_config_value, validate_class_config, validate_text_config,
                                validate_image_conditional_input, validate_class_conditional_input)
from sdmi import leaf as LF
from sdmi.module_glue import EngineHolder, invalidate_module, run_unet


class Unet(nn.Module):
    def __init__(self, im_channels, model_config):
        super().__init__()
        cfg = model_config
        self.im_channels = im_channels
        self.down_channels = cfg["down_channels"]
        self.mid_channels = cfg["mid_channels"]
        self.t_emb_dim = cfg["time_emb_dim"]
        self.down_sample = cfg["down_sample"]
        self.num_down_layers = cfg["num_down_layers"]
        self.num_mid_layers = cfg["num_mid_layers"]
        self.num_up_layers = cfg["num_up_layers"]
        self.attns = cfg["attn_down"]
        self.norm_channels = cfg["norm_channels"]
        self.num_heads = cfg["num_heads"]
        self.conv_out_channels = cfg["conv_out_channels"]
        assert self.mid_channels[0] == self.down_channels[-1]
        assert self.mid_channels[-1] == self.down_channels[-2]
        assert len(self.down_sample) == len(self.down_channels) - 1
        assert len(self.attns) == len(self.down_channels) - 1

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
                self.image_cond = True
                ic = self.condition_config["image_condition_config"]
                self.im_cond_input_ch = ic["image_condition_input_channels"]
                self.im_cond_output_ch = ic["image_condition_output_channels"]
        if self.class_cond:
            self.class_emb = nn.Embedding(self.num_classes, self.t_emb_dim)
        if self.image_cond:
            self.cond_conv_in = nn.Conv2d(self.im_cond_input_ch, self.im_cond_output_ch, kernel_size=1, bias=False)
            self.conv_in_concat = nn.Conv2d(im_channels + self.im_cond_output_ch, self.down_channels[0], 3, padding=1)
        else:
            self.conv_in = nn.Conv2d(im_channels, self.down_channels[0], kernel_size=3, padding=1)
        self.cond = self.text_cond or self.image_cond or self.class_cond
        self.t_proj = nn.Sequential(nn.Linear(self.t_emb_dim, self.t_emb_dim), nn.SiLU(),
                                    nn.Linear(self.t_emb_dim, self.t_emb_dim))
        self.up_sample = list(reversed(self.down_sample))
        dc = self.down_channels
        common = dict(num_heads=self.num_heads, norm_channels=self.norm_channels, cross_attn=self.text_cond,
                      context_dim=self.text_embed_dim)
        self.downs = nn.ModuleList([DownBlock(dc[i], dc[i + 1], self.t_emb_dim, down_sample=self.down_sample[i],
                                              num_layers=self.num_down_layers, attn=self.attns[i], **common)
                                    for i in range(len(dc) - 1)])
        mc = self.mid_channels
        self.mids = nn.ModuleList([MidBlock(mc[i], mc[i + 1], self.t_emb_dim, num_layers=self.num_mid_layers, **common)
                                   for i in range(len(mc) - 1)])
        self.ups = nn.ModuleList([UpBlockUnet(dc[i] * 2, dc[i - 1] if i != 0 else self.conv_out_channels,
                                              self.t_emb_dim, up_sample=self.down_sample[i],
                                              num_layers=self.num_up_layers, **common)
                                  for i in reversed(range(len(dc) - 1))])
        self.norm_out = nn.GroupNorm(self.norm_channels, self.conv_out_channels)
        self.conv_out = nn.Conv2d(self.conv_out_channels, im_channels, kernel_size=3, padding=1)
        self._sdmi = EngineHolder(self, cfg, "cond")

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
        return run_unet(self, self._sdmi, x, t, text, mask, klass)

    def _sdmi_engine_ok(self):
        return LF.engine_ok(self, (Unet, DownBlock, MidBlock, UpBlockUnet))

    def sdmi_invalidate(self):
        """Repack the bf16 weights at the next forward (after writing parameters through `.data`)."""
        invalidate_module(self)

    def _leaf_forward(self, x, t, text, mask, klass):
        """unet_cond_base.py:131-183, leaf by leaf (sdmi.leaf.call)."""
        if self.image_cond:
            im_cond = LF.resize_nearest(mask.float(), x.shape[-2:])
            im_cond = LF.call(self.cond_conv_in, im_cond)
            assert im_cond.shape[-2:] == x.shape[-2:]
            out = LF.call(self.conv_in_concat, LF.cat_channels([x, im_cond]))
        else:
            out = LF.call(self.conv_in, x)
        t_emb = LF.call(self.t_proj, LF.time_embedding(t, x.shape[0], self.t_emb_dim, x.device))
        if self.class_cond:
            t_emb = t_emb + LF.class_embed(self.class_emb, klass)
        return _leaf_body(self, out, t_emb, text)


def _leaf_body(self, out, t_emb, context):
    down_outs = []
    for down in self.downs:
        down_outs.append(out)
        out = down(out, t_emb, context)
    for mid in self.mids:
        out = mid(out, t_emb, context)
    for up in self.ups:
        out = up(out, down_outs.pop(), t_emb, context)
    if type(self.norm_out) is torch.nn.GroupNorm:
        out = LF.group_norm(self.norm_out, out, silu=True)
    else:
        out = LF.call(torch.nn.SiLU(), self.norm_out(out))
    return LF.call(self.conv_out, out)
