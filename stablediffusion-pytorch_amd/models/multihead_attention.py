"""Drop-in mirror of the reference's models/multihead_attention.py (CustomMultiheadAttention, :10-39):
separate q/k/v/out projections with nn.Linear default initialisation. Used by the DiT text
cross-attention; the compute runs inside sdmi.dit_engine (q GEMM, packed k|v GEMM of the projected
context, fused flash attention, out GEMM). On its own it runs multihead_attention.py:41-80 with the projections
on the HIP leaf path and the flash kernel for softmax(q k^T * scaling) v (no masks; dropout 0)."""
import math

import torch
import torch.nn as nn

from sdmi import leaf as LF


class CustomMultiheadAttention(nn.Module):
    def __init__(self, embed_dim, num_heads, dropout=0.0, bias=True, batch_first=False):
        super().__init__()
        if embed_dim % num_heads != 0:
            raise ValueError("embed_dim must be divisible by num_heads")
        self.embed_dim = embed_dim
        self.num_heads = num_heads
        self.head_dim = embed_dim // num_heads
        self.batch_first = batch_first
        self.q_proj = nn.Linear(embed_dim, embed_dim, bias=bias)
        self.k_proj = nn.Linear(embed_dim, embed_dim, bias=bias)
        self.v_proj = nn.Linear(embed_dim, embed_dim, bias=bias)
        self.out_proj = nn.Linear(embed_dim, embed_dim, bias=bias)
        self.dropout = nn.Dropout(dropout) if dropout > 0.0 else nn.Identity()
        self.scaling = 1.0 / math.sqrt(self.head_dim)

    def forward(self, query, key=None, value=None, attn_mask=None, key_padding_mask=None, need_weights=True,
                average_attn_weights=True):
        if attn_mask is not None or key_padding_mask is not None:
            raise NotImplementedError("HIP attention: attention masks are not supported")
        if not isinstance(self.dropout, nn.Identity) and self.training:
            raise NotImplementedError("HIP attention: attention dropout is not supported")
        key = query if key is None else key
        value = key if value is None else value
        if not self.batch_first:
            query, key, value = (t.transpose(0, 1) for t in (query, key, value))
        q, k, v = LF.call(self.q_proj, query), LF.call(self.k_proj, key), LF.call(self.v_proj, value)
        out = LF.call(self.out_proj, LF.attention_core(q, k, v, self.num_heads))
        if not self.batch_first:
            out = out.transpose(0, 1)
        weights = None
        if need_weights:  # the attention map itself (a diagnostic output the flash kernel never materialises)
            weights = LF.attention_map(q, k, self.num_heads, self.scaling, average_attn_weights)
        return out, weights
