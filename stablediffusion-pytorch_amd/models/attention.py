"""Drop-in mirror of the reference's models/attention.py (DiT self-attention, attention.py:7-78).

Parameter holder with the reference's attribute names, shapes and initialisation (qkv_proj packed as
(3 * heads * head_dim, hidden), output_proj = Sequential(Linear)); the compute (one QKV GEMM, the fused
flash-attention kernel with the d^-0.5 scale, the output GEMM) runs inside sdmi.dit_engine for the whole DIT;
called on its own (or inside a DIT with a swapped leaf) it composes its leaves like attention.py:33-78 on the
HIP per-op path (sdmi.leaf).
"""
import torch.nn as nn

from sdmi import leaf as LF


class Attention(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.n_heads = config["num_heads"]
        self.hidden_size = config["hidden_size"]
        self.head_dim = config["head_dim"]
        self.att_dim = self.n_heads * self.head_dim
        self.qkv_proj = nn.Linear(self.hidden_size, 3 * self.att_dim, bias=True)
        self.output_proj = nn.Sequential(nn.Linear(self.att_dim, self.hidden_size))
        nn.init.xavier_uniform_(self.qkv_proj.weight)
        nn.init.constant_(self.qkv_proj.bias, 0)
        nn.init.xavier_uniform_(self.output_proj[0].weight)
        nn.init.constant_(self.output_proj[0].bias, 0)

    def forward(self, x):
        q, k, v = LF.call(self.qkv_proj, x).split(self.att_dim, dim=-1)
        return LF.call(self.output_proj, LF.attention_core(q, k, v, self.n_heads))
