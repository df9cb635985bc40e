"""Drop-in unconditional UNet (reference models/unet_base.py:7-100) on the MI355X HIP path.

Same constructor / forward(x, t) / state-dict keys as the reference (its registration order puts
t_proj before conv_in, unet_base.py:33-39); compute runs in sdmi.unet_engine."""
import torch.nn as nn

from models.blocks import DownBlock, MidBlock, UpBlockUnet, get_time_embedding  # noqa: F401
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
        self.t_proj = nn.Sequential(nn.Linear(self.t_emb_dim, self.t_emb_dim), nn.SiLU(),
                                    nn.Linear(self.t_emb_dim, self.t_emb_dim))
        self.up_sample = list(reversed(self.down_sample))
        self.conv_in = nn.Conv2d(im_channels, self.down_channels[0], kernel_size=3, padding=1)
        dc, mc = self.down_channels, self.mid_channels
        common = dict(num_heads=self.num_heads, norm_channels=self.norm_channels)
        self.downs = nn.ModuleList([DownBlock(dc[i], dc[i + 1], self.t_emb_dim, down_sample=self.down_sample[i],
                                              num_layers=self.num_down_layers, attn=self.attns[i], **common)
                                    for i in range(len(dc) - 1)])
        self.mids = nn.ModuleList([MidBlock(mc[i], mc[i + 1], self.t_emb_dim, num_layers=self.num_mid_layers, **common)
                                   for i in range(len(mc) - 1)])
        self.ups = nn.ModuleList([UpBlockUnet(dc[i] * 2, dc[i - 1] if i != 0 else self.conv_out_channels,
                                              self.t_emb_dim, up_sample=self.down_sample[i],
                                              num_layers=self.num_up_layers, **common)
                                  for i in reversed(range(len(dc) - 1))])
        self.norm_out = nn.GroupNorm(self.norm_channels, self.conv_out_channels)
        self.conv_out = nn.Conv2d(self.conv_out_channels, im_channels, kernel_size=3, padding=1)
        self._sdmi = EngineHolder(self, cfg, "uncond")

    def forward(self, x, t):
        if getattr(self, "sdmi_leaf_path", False) or not self._sdmi_engine_ok():
            # a swapped leaf: unet_base.py:68-100 leaf by leaf
            from models.unet_cond_base import _leaf_body
            out = LF.call(self.conv_in, x)
            t_emb = LF.call(self.t_proj, LF.time_embedding(t, x.shape[0], self.t_emb_dim, x.device))
            return _leaf_body(self, out, t_emb, None)
        return run_unet(self, self._sdmi, x, t)

    def _sdmi_engine_ok(self):
        return LF.engine_ok(self, (Unet, DownBlock, MidBlock, UpBlockUnet))

    def sdmi_invalidate(self):
        """Repack the bf16 weights at the next forward (after writing parameters through `.data`)."""
        invalidate_module(self)
