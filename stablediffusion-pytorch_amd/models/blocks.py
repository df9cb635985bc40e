"""Drop-in mirror of the reference's models/blocks.py module surface.

The blocks have the same attribute names, leaf module types (nn.GroupNorm, nn.Conv2d, nn.ConvTranspose2d,
nn.Linear, nn.MultiheadAttention) and default initialisation as the reference (blocks.py:27-499), so state dicts
and reference checkpoints load unchanged and a layer-swap tool that replaces exact nn.Conv2d / nn.Linear leaves
still finds them. A whole UNet / VQVAE whose leaves are all exact torch types runs as one fused schedule (the
engines of sdmi); a block called on its own, or any block of a model with a swapped leaf, runs the forwards below:
the reference's composition (blocks.py:111-146, 225-267, 343-370, 461-499) with every leaf executed by
sdmi.leaf.call -- exact torch types on the HIP per-op kernels, swapped layers through their own forward.
"""
import torch
import torch.nn as nn

from sdmi import leaf as LF


def get_time_embedding(time_steps, temb_dim):
    """Sinusoidal embedding (reference blocks.py:5-24): [sin(t / 10000^(i/h)), cos(...)], h = d/2.
    Host-side API mirror; inside the UNet the same embedding is computed by sdmi_time_embedding."""
    assert temb_dim % 2 == 0, "time embedding dimension must be divisible by 2"
    half = temb_dim // 2
    freq = 10000 ** (torch.arange(0, half, dtype=torch.float32, device=time_steps.device) / half)
    arg = time_steps[:, None].repeat(1, half) / freq
    return torch.cat([torch.sin(arg), torch.cos(arg)], dim=-1)


def _norm_silu_conv(norm_channels, cin, cout):
    return nn.Sequential(nn.GroupNorm(norm_channels, cin), nn.SiLU(), nn.Conv2d(cin, cout, 3, 1, 1))


def _add_resnets(m, n, cin, cout, t_emb_dim, norm_channels):
    m.resnet_conv_first = nn.ModuleList([_norm_silu_conv(norm_channels, cin if i == 0 else cout, cout) for i in range(n)])
    if t_emb_dim is not None:
        m.t_emb_layers = nn.ModuleList([nn.Sequential(nn.SiLU(), nn.Linear(t_emb_dim, cout)) for _ in range(n)])
    m.resnet_conv_second = nn.ModuleList([_norm_silu_conv(norm_channels, cout, cout) for _ in range(n)])


def _add_attention(m, n, cout, num_heads, norm_channels):
    m.attention_norms = nn.ModuleList([nn.GroupNorm(norm_channels, cout) for _ in range(n)])
    m.attentions = nn.ModuleList([nn.MultiheadAttention(cout, num_heads, batch_first=True) for _ in range(n)])


def _add_cross(m, n, cout, num_heads, norm_channels, context_dim):
    assert context_dim is not None, "Context Dimension must be passed for cross attention"
    m.cross_attention_norms = nn.ModuleList([nn.GroupNorm(norm_channels, cout) for _ in range(n)])
    m.cross_attentions = nn.ModuleList([nn.MultiheadAttention(cout, num_heads, batch_first=True) for _ in range(n)])
    m.context_proj = nn.ModuleList([nn.Linear(context_dim, cout) for _ in range(n)])


def _add_residual(m, n, cin, cout):
    m.residual_input_conv = nn.ModuleList([nn.Conv2d(cin if i == 0 else cout, cout, 1) for i in range(n)])


def _resnet(blk, i, x, t_emb):
    """GN-SiLU-conv, + t_emb_layers(t_emb) per channel, GN-SiLU-conv, + 1x1 residual conv (blocks.py:114-120)."""
    out = LF.call(blk.resnet_conv_first[i], x)
    if blk.t_emb_dim is not None:
        out = out + LF.call(blk.t_emb_layers[i], t_emb)[:, :, None, None]
    out = LF.call(blk.resnet_conv_second[i], out)
    return out + LF.call(blk.residual_input_conv[i], x)


def _attend(norm, attn, out, context=None, proj=None):
    """out + attention(GroupNorm(out) as tokens [, context_proj(context)]) (blocks.py:122-142)."""
    B, C, h, w = out.shape
    a = LF.call(norm, out.reshape(B, C, h * w)).transpose(1, 2)
    if proj is None:
        o, _ = LF.call(attn, a, a, a)
    else:
        cp = LF.call(proj, context)
        o, _ = LF.call(attn, a, cp, cp)
    return out + o.transpose(1, 2).reshape(B, C, h, w)


def _cross(blk, i, out, x, context):
    assert context is not None, "context cannot be None if cross attention layers are used"
    assert len(context.shape) == 3, "Context shape does not match B,_,CONTEXT_DIM"
    assert context.shape[0] == x.shape[0] and context.shape[-1] == blk.context_dim, \
        "Context shape does not match B,_,CONTEXT_DIM"
    return _attend(blk.cross_attention_norms[i], blk.cross_attentions[i], out, context, blk.context_proj[i])


class _ParamBlock(nn.Module):
    pass


class DownBlock(_ParamBlock):
    """resnet x num_layers (+ self-attention, + cross-attention), then Conv(4, 2, 1) (blocks.py:27-146)."""

    def __init__(self, in_channels, out_channels, t_emb_dim, down_sample, num_heads, num_layers, attn, norm_channels,
                 cross_attn=False, context_dim=None):
        super().__init__()
        self.num_layers, self.down_sample, self.attn = num_layers, down_sample, attn
        self.context_dim, self.cross_attn, self.t_emb_dim = context_dim, cross_attn, t_emb_dim
        _add_resnets(self, num_layers, in_channels, out_channels, t_emb_dim, norm_channels)
        if attn:
            _add_attention(self, num_layers, out_channels, num_heads, norm_channels)
        if cross_attn:
            _add_cross(self, num_layers, out_channels, num_heads, norm_channels, context_dim)
        _add_residual(self, num_layers, in_channels, out_channels)
        self.down_sample_conv = nn.Conv2d(out_channels, out_channels, 4, 2, 1) if down_sample else nn.Identity()

    def forward(self, x, t_emb=None, context=None):
        out = x
        for i in range(self.num_layers):
            out = _resnet(self, i, out, t_emb)
            if self.attn:
                out = _attend(self.attention_norms[i], self.attentions[i], out)
            if self.cross_attn:
                out = _cross(self, i, out, x, context)
        return LF.call(self.down_sample_conv, out)


class MidBlock(_ParamBlock):
    """resnet, then num_layers x (self-attention, [cross-attention], resnet) (blocks.py:149-267)."""

    def __init__(self, in_channels, out_channels, t_emb_dim, num_heads, num_layers, norm_channels, cross_attn=None,
                 context_dim=None):
        super().__init__()
        self.num_layers, self.t_emb_dim, self.context_dim, self.cross_attn = num_layers, t_emb_dim, context_dim, cross_attn
        _add_resnets(self, num_layers + 1, in_channels, out_channels, t_emb_dim, norm_channels)
        _add_attention(self, num_layers, out_channels, num_heads, norm_channels)
        if cross_attn:
            _add_cross(self, num_layers, out_channels, num_heads, norm_channels, context_dim)
        _add_residual(self, num_layers + 1, in_channels, out_channels)

    def forward(self, x, t_emb=None, context=None):
        out = _resnet(self, 0, x, t_emb)
        for i in range(self.num_layers):
            out = _attend(self.attention_norms[i], self.attentions[i], out)
            if self.cross_attn:
                out = _cross(self, i, out, x, context)
            out = _resnet(self, i + 1, out, t_emb)
        return out


class UpBlock(_ParamBlock):
    """VQVAE decoder block: ConvTranspose(4, 2, 1) of the full input, num_layers x (resnet, [self-attn])
    (blocks.py:270-370; no skip concatenation)."""

    def __init__(self, in_channels, out_channels, t_emb_dim, up_sample, num_heads, num_layers, attn, norm_channels):
        super().__init__()
        self.num_layers, self.up_sample, self.t_emb_dim, self.attn = num_layers, up_sample, t_emb_dim, attn
        _add_resnets(self, num_layers, in_channels, out_channels, t_emb_dim, norm_channels)
        if attn:
            _add_attention(self, num_layers, out_channels, num_heads, norm_channels)
        _add_residual(self, num_layers, in_channels, out_channels)
        self.up_sample_conv = nn.ConvTranspose2d(in_channels, in_channels, 4, 2, 1) if up_sample else nn.Identity()

    def forward(self, x, out_down=None, t_emb=None):
        x = LF.call(self.up_sample_conv, x)
        if out_down is not None:
            x = LF.cat_channels([x, out_down])
        out = x
        for i in range(self.num_layers):
            out = _resnet(self, i, out, t_emb)
            if self.attn:
                out = _attend(self.attention_norms[i], self.attentions[i], out)
        return out


class UpBlockUnet(_ParamBlock):
    """ConvTranspose(4, 2, 1) of the lower half, concat skip, num_layers x (resnet, self-attn, [cross])
    (blocks.py:373-499)."""

    def __init__(self, in_channels, out_channels, t_emb_dim, up_sample, num_heads, num_layers, norm_channels,
                 cross_attn=False, context_dim=None):
        super().__init__()
        self.num_layers, self.up_sample, self.t_emb_dim = num_layers, up_sample, t_emb_dim
        self.cross_attn, self.context_dim = cross_attn, context_dim
        _add_resnets(self, num_layers, in_channels, out_channels, t_emb_dim, norm_channels)
        _add_attention(self, num_layers, out_channels, num_heads, norm_channels)
        if cross_attn:
            _add_cross(self, num_layers, out_channels, num_heads, norm_channels, context_dim)
        _add_residual(self, num_layers, in_channels, out_channels)
        self.up_sample_conv = (nn.ConvTranspose2d(in_channels // 2, in_channels // 2, 4, 2, 1) if up_sample
                               else nn.Identity())

    def forward(self, x, out_down=None, t_emb=None, context=None):
        x = LF.call(self.up_sample_conv, x)
        if out_down is not None:
            x = LF.cat_channels([x, out_down])
        out = x
        for i in range(self.num_layers):
            out = _resnet(self, i, out, t_emb)
            out = _attend(self.attention_norms[i], self.attentions[i], out)
            if self.cross_attn:
                out = _cross(self, i, out, x, context)
        return out
