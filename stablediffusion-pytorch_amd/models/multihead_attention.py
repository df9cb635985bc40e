"""Drop-in mirror of the reference's models/multihead_attention.py (CustomMultiheadAttention, :10-39):
separate q/k/v/out projections with nn.Linear default initialisation. Used by the DiT text
cross-attention; the compute runs inside sdmi.dit_engine (q GEMM, packed k|v GEMM of the projected
context, fused flash attention, out GEMM)."""
import math

import torch.nn as nn


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

    def forward(self, *args, **kwargs):
        raise NotImplementedError("CustomMultiheadAttention is a parameter holder; run the whole DIT (HIP engine)")
