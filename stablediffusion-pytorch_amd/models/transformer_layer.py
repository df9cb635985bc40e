"""Drop-in mirror of the reference's models/transformer_layer.py (TransformerLayer, :6-78).

Parameter holder with the reference's attribute names (att_norm / ff_norm / cross_attn_norm are
affine-free LayerNorms, attn_block, mlp_block = Linear-ReLU-Linear, optional cross_attn_block +
context_proj, adaptive_norm_layer = ReLU-Linear(6*hidden)) and initialisation (xavier MLP, zero
adaLN). The forward of every layer runs inside sdmi.dit_engine: LayerNorm + adaLN modulation and the
gated residual adds are fused row kernels, the Linears are MFMA GEMMs, attention is the flash kernel.
Called on its own (or in a DIT with a swapped leaf) it runs transformer_layer.py:80-106 leaf by leaf (sdmi.leaf)."""
import torch.nn as nn

from sdmi import leaf as LF

from models.attention import Attention
from models.multihead_attention import CustomMultiheadAttention


class TransformerLayer(nn.Module):
    def __init__(self, config, *, cross_attn=False, context_dim=None):
        super().__init__()
        self.hidden_size = config["hidden_size"]
        self.cross_attn = cross_attn
        self.context_dim = context_dim
        ff_hidden_dim = 4 * self.hidden_size
        self.att_norm = nn.LayerNorm(self.hidden_size, elementwise_affine=False, eps=1E-6)
        self.attn_block = Attention(config)
        self.ff_norm = nn.LayerNorm(self.hidden_size, elementwise_affine=False, eps=1E-6)
        self.mlp_block = nn.Sequential(nn.Linear(self.hidden_size, ff_hidden_dim), nn.ReLU(),
                                       nn.Linear(ff_hidden_dim, self.hidden_size))
        if self.cross_attn:
            assert self.context_dim is not None, "Context dimension must be provided for cross attention"
            self.cross_attn_norm = nn.LayerNorm(self.hidden_size, elementwise_affine=False, eps=1E-6)
            self.cross_attn_block = CustomMultiheadAttention(self.hidden_size, config["num_heads"], batch_first=True)
            self.context_proj = nn.Linear(self.context_dim, self.hidden_size)
        self.adaptive_norm_layer = nn.Sequential(nn.ReLU(), nn.Linear(self.hidden_size, 6 * self.hidden_size, bias=True))
        nn.init.xavier_uniform_(self.mlp_block[0].weight)
        nn.init.constant_(self.mlp_block[0].bias, 0)
        nn.init.xavier_uniform_(self.mlp_block[-1].weight)
        nn.init.constant_(self.mlp_block[-1].bias, 0)
        nn.init.constant_(self.adaptive_norm_layer[-1].weight, 0)
        nn.init.constant_(self.adaptive_norm_layer[-1].bias, 0)
        if self.cross_attn:
            nn.init.xavier_uniform_(self.context_proj.weight)
            nn.init.constant_(self.context_proj.bias, 0)

    def forward(self, x, condition, context=None):
        (pre_attn_shift, pre_attn_scale, post_attn_scale, pre_mlp_shift, pre_mlp_scale,
         post_mlp_scale) = LF.call(self.adaptive_norm_layer, condition).chunk(6, dim=1)
        out = x
        # adaLN modulation and gated residuals on the leaf-glue kernels (sdmi_modulate_fwd / _bwd)
        h = LF.modulate(LF.call(self.att_norm, out), pre_attn_scale, pre_attn_shift)
        out = LF.modulate(self.attn_block(h), post_attn_scale, r=out, alpha=0.0)
        if self.cross_attn and context is not None:
            ctx = LF.call(self.context_proj, context)
            o, _ = self.cross_attn_block(LF.call(self.cross_attn_norm, out), ctx, ctx, need_weights=False)
            out = out + o
        h = LF.modulate(LF.call(self.ff_norm, out), pre_mlp_scale, pre_mlp_shift)
        return LF.modulate(LF.call(self.mlp_block, h), post_mlp_scale, r=out, alpha=0.0)
