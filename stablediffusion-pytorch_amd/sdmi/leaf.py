"""Leaf-module path: the reference's layers callable one at a time on the HIP kernels.

The whole-network engines (sdmi.unet_engine / vqvae_train / dit_engine) run a model as one schedule only while
every leaf of it is still an exact torch type (nn.Conv2d, nn.Linear, nn.GroupNorm, ...). The reference's CIM
stack swaps leaves by exact type -- ProgressiveTrain.convert_to_layers replaces nn.Conv2d / nn.Linear with its
quantised layers and re-uses the Parameter (`new.weight = module.weight`,
cim_qn_train/progressive_qn_train.py:614, 638-640) -- and a caller may also run a block on its own. Then the
blocks compose their leaves exactly like the reference's forwards (models/blocks.py:111-146, 225-267, 343-370,
461-499), and `call(module, ...)` runs each leaf: an exact torch type on the HIP per-op path below, anything else
(a swapped layer) through its own forward.

Per-op path: each leaf is one autograd Function over NCHW / row-major fp32 torch tensors (the interface a
swapped layer expects); inside, activations are converted to NHWC bf16 for the MFMA implicit-GEMM / GroupNorm /
attention kernels, results come back as fp32, and the backward runs the same kernels' data / weight gradients.
Packed bf16 weights are cached per module and repacked when the parameter's version changes. The glue between
leaves that is more than an add -- mask resize, channel concatenation, the DiT's adaLN modulation and gated residuals,
need_weights attention maps -- runs on csrc/leafops.hip; plain residual adds stay torch, as in the reference's
block code."""
import weakref

import torch
import torch.nn as nn

from . import _lib
from . import kernels as K
from .unet_engine import PackPlan


def _r8(n):
    return (n + 7) // 8 * 8


def _nhwc(x, ld):
    """(B, C, *spatial) fp32 -> NHWC bf16 [B*P, ld] (channels >= C zero)."""
    x = x.float().contiguous()
    B, C = x.shape[0], x.shape[1]
    P = x[0, 0].numel() if x.dim() > 2 else 1
    out = torch.empty(B * P, ld, dtype=torch.bfloat16, device=x.device)
    _lib.check(_lib.lib().sdmi_nchw_to_nhwc_bf16(x.data_ptr(), B, C, P, out.data_ptr(), ld, K._stream()), "to_nhwc")
    return out


def _nchw(y, ld, shape):
    """NHWC [B*P, ld] (bf16 or fp32) -> fp32 tensor of `shape` = (B, C, *spatial)."""
    B, C = shape[0], shape[1]
    P = 1
    for s in shape[2:]:
        P *= s
    out = torch.empty(shape, dtype=torch.float32, device=y.device)
    _lib.check(_lib.lib().sdmi_nhwc_to_nchw(y.data_ptr(), 1 if y.dtype == torch.float32 else 0, ld, B, C, P,
                                            out.data_ptr(), K._stream()), "to_nchw")
    return out


def _rows(x, ld):
    """(M, Kd) fp32 -> bf16 [M, ld] (columns >= Kd zero)."""
    M, Kd = x.shape
    return _nhwc(x.reshape(M, Kd, 1), ld)


def _unrows(y, ld, M, N):
    return _nchw(y, ld, (M, N, 1)).reshape(M, N)


# ---- packed weights, cached per module ----------------------------------------------------------------------------
_PACKS = weakref.WeakKeyDictionary()


def _packed(mod, w, build):
    """PackPlan of `w` built by build(pk, w) once per (module, storage). Repacked on every grad-enabled call (updates
    through `.data` keep the version counter, see module_glue.EngineHolder.refresh) and, under torch.no_grad, when
    w's version changed or invalidate_packs(mod) was called."""
    ent = _PACKS.get(mod)
    if ent is None or ent["ptr"] != w.data_ptr():
        pk = PackPlan(w.device)
        build(pk, w.detach())
        pk.finalize()
        ent = {"ptr": w.data_ptr(), "ver": None, "pk": pk}
        _PACKS[mod] = ent
    if torch.is_grad_enabled() or ent["ver"] != w._version:
        ent["pk"].run()
        ent["ver"] = w._version
    return ent["pk"]


def invalidate_packs(mod=None):
    """Drop the cached pack state of `mod`'s leaves (every leaf when mod is None): the next forward repacks."""
    if mod is None:
        for ent in _PACKS.values():
            ent["ver"] = None
        return
    for m in mod.modules():
        ent = _PACKS.get(m)
        if ent is not None:
            ent["ver"] = None


def _pack_conv(mod):
    w = mod.weight
    O, I, KH, KW = w.shape
    Ip, Op = _r8(I), _r8(O)

    def build(pk, w):
        pk.add("f", w, O, I, Ip, KH, KW, I * KH * KW, KH * KW, KW, 1, rows=Op)
        if mod.stride[0] == 1:  # stride-1 data gradient: flipped taps, transposed
            pk.add_transpose("d", "f", O, I, KH * KW, [KH * KW - 1 - t for t in range(KH * KW)], Ip, rows=Ip, opad=Op)
        else:  # k4 s2 p1: four 2x2 sub-pixel phases of the data gradient
            for ph in range(2):
                for pw in range(2):
                    pk.add_transpose(f"d{ph}{pw}", "f", O, I, 4,
                                     [(3 - ph - 2 * a) * 4 + (3 - pw - 2 * b) for a in range(2) for b in range(2)], Ip,
                                     rows=Ip, opad=Op)
    return _packed(mod, w, build)


def _pack_convT(mod):
    w = mod.weight  # (Cx, Cy, 4, 4)
    Cx, Cy = w.shape[0], w.shape[1]

    def build(pk, w):
        pk.add("d", w, Cx, Cy, Cy, 4, 4, Cy * 16, 16, 4, 1)
        for ph in range(2):
            for pw in range(2):
                pk.add_transpose(f"f{ph}{pw}", "d", Cx, Cy, 4,
                                 [(3 - ph - 2 * a) * 4 + (3 - pw - 2 * b) for a in range(2) for b in range(2)], Cy)
    return _packed(mod, w, build)


def _pack_linear(mod, w=None):
    w = mod.weight if w is None else w
    N, Kd = w.shape

    def build(pk, w):
        pk.add("f", w, N, Kd, _r8(Kd), 1, 1, Kd, 1, 0, 0, rows=_r8(N))
    return _packed(mod, w, build)


# ---- Conv2d -------------------------------------------------------------------------------------------------------
class _Conv2d(torch.autograd.Function):
    @staticmethod
    def forward(ctx, mod, x, weight, bias):
        B, I, H, W = x.shape
        O, _, KH, KW = weight.shape
        s, p = mod.stride[0], mod.padding[0]
        Ip, Op = _r8(I), _r8(O)
        pk = _pack_conv(mod)
        xin = _nhwc(x, Ip)
        OH, OW = (H + 2 * p - KH) // s + 1, (W + 2 * p - KW) // s + 1
        y = torch.empty(B * OH * OW, Op, dtype=torch.float32, device=x.device)
        K.conv_fwd(xin, B, H, W, Ip, Ip, pk.view("f"), Op, KH, KW, s, p, y, Op, bias=bias, n_store=O)
        ctx.mod, ctx.xin, ctx.geo = mod, xin, (B, I, H, W, O, KH, KW, s, p, OH, OW)
        ctx.has_bias = bias is not None
        return _nchw(y, Op, (B, O, OH, OW))

    @staticmethod
    def backward(ctx, dy):
        B, I, H, W, O, KH, KW, s, p, OH, OW = ctx.geo
        mod = ctx.mod
        Ip, Op = _r8(I), _r8(O)
        pk = _pack_conv(mod)
        dyb = _nhwc(dy, Op)
        dw = torch.empty_like(mod.weight)
        db = torch.empty_like(mod.bias) if ctx.has_bias else None
        K.conv_wgrad(dyb, Op, ctx.xin, B, H, W, Ip, Ip, Op, KH, KW, s, p, dw, OH, OW, cvalid=I, m_store=O,
                     bias_grad=db)
        dx = None
        if ctx.needs_input_grad[1]:
            dxf = torch.empty(B * H * W, Ip, dtype=torch.float32, device=dy.device)
            if s == 1:
                K.conv_fwd(dyb, B, OH, OW, Op, Op, pk.view("d"), Ip, KH, KW, 1, KH - 1 - p, dxf, Ip)
            else:
                K.conv_dgrad_phases(dyb, B, H, W, Op, Op, [pk.view(f"d{a}{b}") for a in range(2) for b in range(2)],
                                    Ip, dxf, Ip)
            dx = _nchw(dxf, Ip, (B, I, H, W))
        ctx.xin = None
        return None, dx, dw, db


def conv2d(mod, x):
    s, p = mod.stride, mod.padding
    ok = (mod.groups == 1 and tuple(mod.dilation) == (1, 1) and s[0] == s[1] and p[0] == p[1]
          and mod.padding_mode == "zeros" and not isinstance(p, str) and x.dim() == 4
          and (s[0] == 1 and 2 * p[0] == mod.kernel_size[0] - 1 == mod.kernel_size[1] - 1
               or (s[0], p[0], tuple(mod.kernel_size)) == (2, 1, (4, 4))))
    if not ok:
        raise NotImplementedError(f"HIP leaf Conv2d: unsupported geometry {mod}")
    return _Conv2d.apply(mod, x, mod.weight, mod.bias)


# ---- ConvTranspose2d (k4 s2 p1, the reference's up-sampling) ------------------------------------------------------
class _ConvT(torch.autograd.Function):
    @staticmethod
    def forward(ctx, mod, x, weight, bias):
        B, C, H, W = x.shape
        pk = _pack_convT(mod)
        xin = _nhwc(x, C)
        y = torch.empty(B * 4 * H * W, C, dtype=torch.float32, device=x.device)
        K.convT_fwd_phases(xin, B, H, W, C, C, [pk.view(f"f{a}{b}") for a in range(2) for b in range(2)], C, y, C,
                           bias=bias)
        ctx.mod, ctx.xin, ctx.geo, ctx.has_bias = mod, xin, (B, C, H, W), bias is not None
        return _nchw(y, C, (B, C, 2 * H, 2 * W))

    @staticmethod
    def backward(ctx, dy):
        B, C, H, W = ctx.geo
        mod = ctx.mod
        pk = _pack_convT(mod)
        dyb = _nhwc(dy, C)
        dw = torch.empty_like(mod.weight)
        g = K.conv_geom(2 * H, 2 * W, C, C, 4, 4, H, W, 2, 2, -1, -1)
        K.gemm(C, 16 * C, B * H * W, ctx.xin, _lib.A_COLMAJOR, C, dyb, _lib.B_KN_CONV, 0, dw, 16 * C, geom=g,
               perm=(C, 16))
        db = None
        if ctx.has_bias:
            db = torch.empty_like(mod.bias)
            K.chan_sum(dyb, B, 4 * H * W, C, per_c=db)
        dx = None
        if ctx.needs_input_grad[1]:
            dxf = torch.empty(B * H * W, C, dtype=torch.float32, device=dy.device)
            K.conv_fwd(dyb, B, 2 * H, 2 * W, C, C, pk.view("d"), C, 4, 4, 2, 1, dxf, C)
            dx = _nchw(dxf, C, (B, C, H, W))
        ctx.xin = None
        return None, dx, dw, db


def conv_transpose2d(mod, x):
    if (tuple(mod.kernel_size), tuple(mod.stride), tuple(mod.padding)) != ((4, 4), (2, 2), (1, 1)) or \
            mod.in_channels != mod.out_channels or mod.in_channels % 8 or mod.groups != 1 or \
            tuple(mod.output_padding) != (0, 0):
        raise NotImplementedError(f"HIP leaf ConvTranspose2d: unsupported geometry {mod}")
    return _ConvT.apply(mod, x, mod.weight, mod.bias)


# ---- Linear -------------------------------------------------------------------------------------------------------
class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, mod, x, weight, bias):
        N, Kd = weight.shape
        lead = x.shape[:-1]
        x2 = x.reshape(-1, Kd)
        M = x2.shape[0]
        Kp, Np = _r8(Kd), _r8(N)
        pk = _pack_linear(mod, weight)
        xb = _rows(x2, Kp)
        y = torch.empty(M, Np, dtype=torch.float32, device=x.device)
        K.linear(xb, pk.view("f"), y, bias=bias, n_store=N)
        ctx.mod, ctx.xb, ctx.geo, ctx.has_bias = mod, xb, (M, N, Kd, lead), bias is not None
        ctx.weight = weight
        return _unrows(y, Np, M, N).reshape(*lead, N)

    @staticmethod
    def backward(ctx, dy):
        M, N, Kd, lead = ctx.geo
        Kp, Np = _r8(Kd), _r8(N)
        pk = _pack_linear(ctx.mod, ctx.weight)
        dyb = _rows(dy.reshape(M, N), Np)
        db = torch.empty(N, dtype=torch.float32, device=dy.device) if ctx.has_bias else None
        if Kd == Kp:
            dw = torch.empty_like(ctx.weight)
            K.linear_wgrad(dyb, ctx.xb, dw, bias_grad=db, m_store=N)
        else:  # the GEMM's row / column counts are multiples of 8: a padded gradient, then its first Kd columns
            dwp = torch.empty(N, Kp, dtype=torch.float32, device=dy.device)
            K.linear_wgrad(dyb, ctx.xb, dwp, bias_grad=db, m_store=N)
            dw = _unrows(dwp, Kp, N, Kd)
        dx = None
        if ctx.needs_input_grad[1]:
            dxf = torch.empty(M, Kp, dtype=torch.float32, device=dy.device)
            K.linear_dgrad(dyb, pk.view("f"), dxf)
            dx = _unrows(dxf, Kp, M, Kd).reshape(*lead, Kd)
        ctx.xb = None
        return None, dx, dw, db


def linear(mod, x):
    return _Linear.apply(mod, x, mod.weight, mod.bias)


# ---- GroupNorm (+ SiLU) -------------------------------------------------------------------------------------------
class _GroupNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, mod, x, gamma, beta, silu):
        B, C = x.shape[0], x.shape[1]
        P = x[0, 0].numel()
        xb = _nhwc(x, C)
        y = torch.empty(B * P, C, dtype=torch.bfloat16, device=x.device)
        tab = K.gn_fwd(xb, B, P, C, mod.num_groups, gamma, beta, silu, y, eps=mod.eps)
        ctx.save = (xb, tab, gamma, B, P, C, mod.num_groups, silu, x.shape)
        return _nchw(y, C, x.shape)

    @staticmethod
    def backward(ctx, dy):
        xb, tab, gamma, B, P, C, G, silu, shape = ctx.save
        dyb = _nhwc(dy, C)
        dx = torch.empty(B * P, C, dtype=torch.bfloat16, device=dy.device)
        dg = torch.empty(C, dtype=torch.float32, device=dy.device)
        dbeta = torch.empty(C, dtype=torch.float32, device=dy.device)
        K.gn_bwd(xb, dyb, dx, tab, gamma, B, P, C, G, silu, dg, dbeta)
        ctx.save = None
        return None, _nchw(dx, C, shape), dg, dbeta, None


def group_norm(mod, x, silu=False):
    if not mod.affine:
        raise NotImplementedError("HIP leaf GroupNorm: affine=False")
    return _GroupNorm.apply(mod, x, mod.weight, mod.bias, silu)


# ---- SiLU ---------------------------------------------------------------------------------------------------------
class _SiLU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        n = x.numel()
        xb = _rows(x.reshape(n, 1), 1)
        y = torch.empty_like(xb)
        _lib.check(_lib.lib().sdmi_silu(xb.data_ptr(), None, y.data_ptr(), n, K._stream()), "sdmi_silu")
        ctx.xb, ctx.shape = xb, x.shape
        return _unrows(y, 1, n, 1).reshape(x.shape)

    @staticmethod
    def backward(ctx, dy):
        n = dy.numel()
        dyb = _rows(dy.reshape(n, 1), 1)
        dx = torch.empty_like(dyb)
        _lib.check(_lib.lib().sdmi_silu(ctx.xb.data_ptr(), dyb.data_ptr(), dx.data_ptr(), n, K._stream()), "silu")
        ctx.xb = None
        return _unrows(dx, 1, n, 1).reshape(ctx.shape)


# ---- ReLU (fp32) --------------------------------------------------------------------------------------------------
class _ReLU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        x = x.float().contiguous()
        y = torch.empty_like(x)
        _lib.check(_lib.lib().sdmi_relu(x.data_ptr(), None, y.data_ptr(), x.numel(), K._stream()), "sdmi_relu")
        ctx.x = x
        return y

    @staticmethod
    def backward(ctx, dy):
        dy = dy.float().contiguous()
        dx = torch.empty_like(dy)
        _lib.check(_lib.lib().sdmi_relu(ctx.x.data_ptr(), dy.data_ptr(), dx.data_ptr(), dy.numel(), K._stream()),
                   "sdmi_relu")
        ctx.x = None
        return dx


# ---- LayerNorm without affine (the DiT's norms, transformer_layer.py:21-28) ---------------------------------------
class _LayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, eps):
        C = x.shape[-1]
        x2 = x.float().contiguous().reshape(-1, C)
        rows = x2.shape[0]
        N = x.shape[-2] if x.dim() >= 3 else rows  # rows per sample
        y = torch.empty(rows, C, dtype=torch.bfloat16, device=x.device)
        mean = torch.empty(rows, dtype=torch.float32, device=x.device)
        rstd = torch.empty_like(mean)
        _lib.check(_lib.lib().sdmi_ln_mod_fwd(x2.data_ptr(), C, None, 0, None, None, 0, None, None, 0, y.data_ptr(), C,
                                              mean.data_ptr(), rstd.data_ptr(), rows, C, N, eps, 1, K._stream()),
                   "sdmi_ln_mod_fwd")
        ctx.save = (x2, mean, rstd, rows, C, N, x.shape)
        return _unrows(y, C, rows, C).reshape(x.shape)

    @staticmethod
    def backward(ctx, dy):
        x2, mean, rstd, rows, C, N, shape = ctx.save
        dyb = _rows(dy.reshape(rows, C), C)
        dx = torch.empty(rows, C, dtype=torch.float32, device=dy.device)
        _lib.check(_lib.lib().sdmi_ln_mod_bwd(x2.data_ptr(), C, mean.data_ptr(), rstd.data_ptr(), dyb.data_ptr(), C,
                                              None, 0, None, 0, dx.data_ptr(), C, None, None, 0, None, None, 0, None,
                                              0, None, rows, C, N, 1, None, 0, K._stream()), "sdmi_ln_mod_bwd")
        ctx.save = None
        return dx.reshape(shape), None


def layer_norm(mod, x):
    C = x.shape[-1]
    if mod.elementwise_affine or tuple(mod.normalized_shape) != (C,) or C % 8 or C > 512:
        raise NotImplementedError(f"HIP leaf LayerNorm: unsupported {mod}")
    return _LayerNorm.apply(x, mod.eps)


# ---- attention core: softmax(q k^T / sqrt(d)) v over heads (attention.py:41-73, multihead_attention.py:56-67) -----
class _AttnCore(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, heads):
        B, N, E = q.shape
        S = k.shape[1]
        d = E // heads
        qb, kb, vb = (_rows(t.reshape(-1, E), E) for t in (q, k, v))
        o = torch.empty(B * N, E, dtype=torch.bfloat16, device=q.device)
        lse = K.attn_fwd(qb, kb, vb, o, B, heads, N, S, d)
        ctx.save = (qb, kb, vb, o, lse, (B, N, S, E, heads, d))
        return _unrows(o, E, B * N, E).reshape(B, N, E)

    @staticmethod
    def backward(ctx, dy):
        qb, kb, vb, o, lse, (B, N, S, E, H, d) = ctx.save
        dyb = _rows(dy.reshape(B * N, E), E)
        dq, dk, dv = (torch.empty(n, E, dtype=torch.bfloat16, device=dy.device) for n in (B * N, B * S, B * S))
        K.attn_bwd(qb, kb, vb, o, dyb, lse, dq, dk, dv, B, H, N, S, d)
        ctx.save = None
        return (_unrows(dq, E, B * N, E).reshape(B, N, E), _unrows(dk, E, B * S, E).reshape(B, S, E),
                _unrows(dv, E, B * S, E).reshape(B, S, E), None)


def attention_core(q, k, v, heads):
    E = q.shape[-1]
    if E % heads or (E // heads) % 8 or E // heads > 64 or E % 8:
        raise NotImplementedError("HIP attention: head_dim must be a multiple of 8 and <= 64")
    return _AttnCore.apply(q.contiguous(), k.contiguous(), v.contiguous(), heads)


# ---- nn.MultiheadAttention (batch_first, packed in-projection) ----------------------------------------------------
class _MHA(torch.autograd.Function):
    """softmax(q k^T / sqrt(d)) v with nn.MultiheadAttention's packed in_proj / out_proj; q_in (B, N, C),
    kv_in (B, S, C) (the same tensor for self-attention)."""

    @staticmethod
    def forward(ctx, mod, same, q_in, kv_in, w_in, b_in, w_out, b_out):
        B, N, C = q_in.shape
        S = kv_in.shape[1]
        H = mod.num_heads
        d = C // H
        dev = q_in.device
        pin = _pack_linear(mod, w_in)
        pout = _pack_linear(mod.out_proj, w_out)
        Win = pin.view("f")
        a = _rows(q_in.reshape(B * N, C), C)
        o = torch.empty(B * N, C, dtype=torch.bfloat16, device=dev)
        if same:
            qkv = torch.empty(B * N, 3 * C, dtype=torch.bfloat16, device=dev)
            K.linear(a, Win, qkv, bias=b_in)
            q, k, v = qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:]
            c = None
        else:
            c = _rows(kv_in.reshape(B * S, C), C)
            q = torch.empty(B * N, C, dtype=torch.bfloat16, device=dev)
            K.linear(a, Win[:C], q, bias=b_in[:C])
            kv = torch.empty(B * S, 2 * C, dtype=torch.bfloat16, device=dev)
            K.linear(c, Win[C:], kv, bias=b_in[C:])
            k, v = kv[:, :C], kv[:, C:]
        lse = K.attn_fwd(q, k, v, o, B, H, N, S, d)
        y = torch.empty(B * N, C, dtype=torch.float32, device=dev)
        K.linear(o, pout.view("f"), y, bias=b_out)
        ctx.save = (mod, same, a, c, q, k, v, o, lse, w_in, w_out, (B, N, S, C, H, d))
        return y.reshape(B, N, C)

    @staticmethod
    def backward(ctx, dy):
        mod, same, a, c, q, k, v, o, lse, w_in, w_out, (B, N, S, C, H, d) = ctx.save
        dev = dy.device
        pin = _pack_linear(mod, w_in)
        pout = _pack_linear(mod.out_proj, w_out)
        Win = pin.view("f")
        dyb = _rows(dy.reshape(B * N, C), C)
        gWout = torch.empty_like(w_out)
        gbout = torch.empty(C, dtype=torch.float32, device=dev)
        K.linear_wgrad(dyb, o, gWout, bias_grad=gbout)
        do = torch.empty(B * N, C, dtype=torch.bfloat16, device=dev)
        K.linear_dgrad(dyb, pout.view("f"), do)
        gWin = torch.empty_like(w_in)
        gbin = torch.empty(3 * C, dtype=torch.float32, device=dev)
        dq_in = torch.empty(B * N, C, dtype=torch.float32, device=dev)
        dkv_in = None
        if same:
            dqkv = torch.empty(B * N, 3 * C, dtype=torch.bfloat16, device=dev)
            K.attn_bwd(q, k, v, o, do, lse, dqkv[:, :C], dqkv[:, C:2 * C], dqkv[:, 2 * C:], B, H, N, S, d)
            K.linear_wgrad(dqkv, a, gWin, bias_grad=gbin)
            K.linear_dgrad(dqkv, Win, dq_in)
        else:
            dq = torch.empty(B * N, C, dtype=torch.bfloat16, device=dev)
            dkv = torch.empty(B * S, 2 * C, dtype=torch.bfloat16, device=dev)
            K.attn_bwd(q, k, v, o, do, lse, dq, dkv[:, :C], dkv[:, C:], B, H, N, S, d)
            K.linear_wgrad(dq, a, gWin[:C], bias_grad=gbin[:C])
            K.linear_wgrad(dkv, c, gWin[C:], bias_grad=gbin[C:])
            K.linear_dgrad(dq, Win[:C], dq_in)
            dkv_in = torch.empty(B * S, C, dtype=torch.float32, device=dev)
            K.linear_dgrad(dkv, Win[C:], dkv_in)
            dkv_in = dkv_in.reshape(B, S, C)
        ctx.save = None
        return None, None, dq_in.reshape(B, N, C), dkv_in, gWin, gbin, gWout, gbout


def multihead_attention(mod, query, key, value):
    """nn.MultiheadAttention(batch_first=True)(query, key, value) -> (out, None) for self- (q is k is v) and
    cross-attention (k is v), as the reference's blocks call it (blocks.py:128, :140)."""
    C = mod.embed_dim
    if not (mod.batch_first and mod._qkv_same_embed_dim and mod.in_proj_bias is not None and mod.bias_k is None
            and not mod.add_zero_attn and key is value and C % 8 == 0 and (C // mod.num_heads) % 8 == 0
            and C // mod.num_heads <= 64):
        raise NotImplementedError("HIP leaf MultiheadAttention: only the reference's configuration")
    same = query is key
    out = _MHA.apply(mod, same, query.contiguous(), key.contiguous(), mod.in_proj_weight, mod.in_proj_bias,
                     mod.out_proj.weight, mod.out_proj.bias)
    return out, None


# ---- class embedding (unet_cond_base.py:152-155: einsum(class, class_emb.weight)) ---------------------------------
class _ClassEmbed(torch.autograd.Function):
    @staticmethod
    def forward(ctx, mod, klass, weight):
        n, d = weight.shape
        npad = _r8(n)
        B = klass.shape[0]

        def build(pk, w):  # [class (zero rows up to npad)][d]: the B operand (k = class) of the GEMM
            pk.add("kn", w, n, d, d, 1, 1, d, 1, 0, 0, rows=npad)
        pk = _packed(mod, weight, build)
        kb = _rows(klass.float(), npad)
        y = torch.empty(B, d, dtype=torch.float32, device=klass.device)
        K.gemm(B, d, npad, kb, _lib.A_ROWMAJOR, npad, pk.view("kn"), _lib.B_KN, d, y, d)
        ctx.save = (kb, weight, B, n, d)
        return y

    @staticmethod
    def backward(ctx, dy):
        kb, weight, B, n, d = ctx.save
        dyb = _rows(dy, d)
        dw = torch.empty_like(weight)
        K.gemm(_r8(n), d, B, kb, _lib.A_COLMAJOR, _r8(n), dyb, _lib.B_KN, d, dw, d, m_store=n)
        ctx.save = None
        return None, None, dw


def class_embed(mod, klass):
    if type(mod) is not nn.Embedding:
        return torch.einsum("bn,nd->bd", klass.float(), mod.weight)  # a swapped embedding: its own weight
    return _ClassEmbed.apply(mod, klass, mod.weight)


# ---- VQVAE quantiser (vqvae.py:93-126) on its own: sdmi_vq_quantize / sdmi_vq_bwd with identity 1x1 convs ----------
class _Quantize(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, emb):
        B, C, h, w = x.shape
        Kc = emb.shape[0]
        dev = x.device
        P = B * h * w
        z = x.detach().permute(0, 2, 3, 1).reshape(P, C).contiguous()  # NHWC fp32 rows
        eye = torch.eye(C, dtype=torch.float32, device=dev)
        zero = torch.zeros(C, dtype=torch.float32, device=dev)
        zq = torch.empty(B, C, h, w, dtype=torch.float32, device=dev)
        pre = torch.empty_like(zq)
        idx = torch.empty(B, h, w, dtype=torch.int64, device=dev)
        loss = torch.empty(1, dtype=torch.float32, device=dev)
        L = _lib.lib()
        ws = torch.empty(L.sdmi_vq_workspace(P) // 4 + 1, dtype=torch.float32, device=dev)
        _lib.check(L.sdmi_vq_quantize(z.data_ptr(), C, eye.data_ptr(), zero.data_ptr(), emb.data_ptr(), Kc, B, h * w,
                                      C, zq.data_ptr(), idx.data_ptr(), pre.data_ptr(), ws.data_ptr(), loss.data_ptr(),
                                      K._stream()), "sdmi_vq_quantize")
        ctx.save = (z, pre, zq, idx, emb, eye, (B, C, h, w, Kc))
        ctx.mark_non_differentiable(idx)
        return zq, loss[0].clone(), loss[0].clone(), idx

    @staticmethod
    def backward(ctx, dzq, dcb, dcm, _didx):
        z, pre, zq, idx, emb, eye, (B, C, h, w, Kc) = ctx.save
        dev = z.device
        P = B * h * w
        zero = torch.zeros((), device=dev)
        loss_w = torch.stack([(dcb if dcb is not None else zero).float().reshape(()),
                              (dcm if dcm is not None else zero).float().reshape(())])
        dzin = torch.zeros(P, 8, dtype=torch.bfloat16, device=dev)
        dx = torch.empty(P, 8, dtype=torch.bfloat16, device=dev)
        demb = torch.empty_like(emb)
        L = _lib.lib()
        ws = torch.empty(L.sdmi_vq_bwd_workspace() // 4, dtype=torch.float32, device=dev)
        dzq_c = dzq.float().contiguous() if dzq is not None else None
        _lib.check(L.sdmi_vq_bwd(dzin.data_ptr(), 8, zq.data_ptr(), eye.data_ptr(), pre.data_ptr(), idx.data_ptr(),
                                 emb.data_ptr(), Kc, z.data_ptr(), C, eye.data_ptr(), B, h * w, C, 1.0, 1.0,
                                 dx.data_ptr(), 8, ws.data_ptr(), None, None, None, None, demb.data_ptr(),
                                 K._p(dzq_c), loss_w.data_ptr(), K._stream()), "sdmi_vq_bwd")
        ctx.save = None
        return _nchw(dx, 8, (B, C, h, w)), demb


def quantize(embedding, x):
    """VQVAE.quantize (vqvae.py:93-126): (z_q with the straight-through gradient, {'codebook_loss',
    'commitment_loss'}, indices (B, h, w))."""
    zq, cb, cm, idx = _Quantize.apply(x, embedding.weight)
    return zq, {"codebook_loss": cb, "commitment_loss": cm}, idx


# ---- glue between leaves (csrc/leafops.hip): nearest resize, channel concatenation, adaLN modulation, attention map --
def resize_nearest(x, size):
    """F.interpolate(x, size) with the default mode 'nearest' (unet_cond_base.py:132, transformer.py:169) of a
    (B, C, H, W) fp32 tensor. The mask condition is data: no gradient flows to it."""
    if x.requires_grad:
        raise NotImplementedError("HIP leaf resize_nearest: no gradient w.r.t. the resized tensor")
    x = x.float().contiguous()
    B, C, H, W = x.shape
    OH, OW = int(size[0]), int(size[1])
    out = torch.empty(B, C, OH, OW, dtype=torch.float32, device=x.device)
    _lib.check(_lib.lib().sdmi_resize_nearest(x.data_ptr(), B * C, H, W, out.data_ptr(), OH, OW, K._stream()),
               "sdmi_resize_nearest")
    return out


def _chan_copy(src, s0, dst, d0, C):
    B, sC, dC = src.shape[0], src.shape[1], dst.shape[1]
    P = src[0, 0].numel()
    _lib.check(_lib.lib().sdmi_chan_copy(src.data_ptr(), sC, s0, dst.data_ptr(), dC, d0, B, C, P, K._stream()),
               "sdmi_chan_copy")


class _CatChannels(torch.autograd.Function):
    @staticmethod
    def forward(ctx, *xs):
        B, sp = xs[0].shape[0], tuple(xs[0].shape[2:])
        cs = [x.shape[1] for x in xs]
        out = torch.empty(B, sum(cs), *sp, dtype=torch.float32, device=xs[0].device)
        c0 = 0
        for x, c in zip(xs, cs):
            _chan_copy(x, 0, out, c0, c)
            c0 += c
        ctx.cs = cs
        return out

    @staticmethod
    def backward(ctx, dout):
        dout = dout.float().contiguous()
        grads, c0 = [], 0
        for c, need in zip(ctx.cs, ctx.needs_input_grad):
            g = None
            if need:
                g = torch.empty(dout.shape[0], c, *dout.shape[2:], dtype=torch.float32, device=dout.device)
                _chan_copy(dout, c0, g, 0, c)
            grads.append(g)
            c0 += c
        return tuple(grads)


def cat_channels(xs):
    """torch.cat(xs, dim=1) of (B, C_i, *spatial) fp32 tensors (unet_cond_base.py:136, blocks.py:463-464,
    transformer.py:170); its backward splits the gradient with the same kernel."""
    xs = [x.float().contiguous() for x in xs]
    if any(x.shape[0] != xs[0].shape[0] or x.shape[2:] != xs[0].shape[2:] for x in xs):
        raise ValueError("cat_channels: batch and spatial sizes must match")
    return _CatChannels.apply(*xs)


class _Modulate(torch.autograd.Function):
    """y = r + x * (alpha + s[:, None]) + t[:, None] over x (B, N, C); s, t (B, C) rows of stride ls."""

    @staticmethod
    def forward(ctx, x, s, t, r, alpha, ls):
        B, N, C = x.shape
        y = torch.empty_like(x)
        _lib.check(_lib.lib().sdmi_modulate_fwd(x.data_ptr(), K._p(r), s.data_ptr(), K._p(t), ls, float(alpha),
                                                y.data_ptr(), B, N, C, K._stream()), "sdmi_modulate_fwd")
        ctx.save_for_backward(x, s)
        ctx.alpha, ctx.ls, ctx.has_t, ctx.has_r = alpha, ls, t is not None, r is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, s = ctx.saved_tensors
        dy = dy.float().contiguous()
        B, N, C = x.shape
        dev = dy.device
        dx = torch.empty_like(x) if ctx.needs_input_grad[0] else None
        # ds / dt are written with the same row stride as s / t (ls): a (B, ls) buffer, returned as (B, C) views
        ds = torch.zeros(B, ctx.ls, dtype=torch.float32, device=dev) if ctx.needs_input_grad[1] else None
        dt = torch.zeros(B, ctx.ls, dtype=torch.float32, device=dev) if ctx.has_t and ctx.needs_input_grad[2] else None
        _lib.check(_lib.lib().sdmi_modulate_bwd(x.data_ptr(), dy.data_ptr(), s.data_ptr(), ctx.ls, float(ctx.alpha),
                                                K._p(dx), K._p(ds), K._p(dt), B, N, C, K._stream()),
                   "sdmi_modulate_bwd")
        dr = dy if ctx.has_r and ctx.needs_input_grad[3] else None
        return (dx, ds[:, :C] if ds is not None else None, dt[:, :C] if dt is not None else None, dr, None, None)


def modulate(x, s, t=None, r=None, alpha=1.0):
    """(r +) x * (alpha + s.unsqueeze(1)) (+ t.unsqueeze(1)) for x (B, N, C) and per-(sample, channel) s, t (B, C):
    the DiT's adaLN modulation (alpha 1, t = shift) and gated residual (alpha 0, r = the residual stream)."""
    x = x.float().contiguous()
    r = r.float().contiguous() if r is not None else None
    B, N, C = x.shape

    def rows(v):  # (B, C) with unit column stride: pass its row stride; else a compact copy
        return v if v.dtype == torch.float32 and v.stride(1) == 1 else v.float().contiguous()
    s = rows(s)
    t = rows(t) if t is not None else None
    if t is not None and t.stride(0) != s.stride(0):
        s, t = s.contiguous(), t.contiguous()
    if tuple(s.shape) != (B, C) or (t is not None and tuple(t.shape) != (B, C)):
        raise ValueError("modulate: s / t must be (B, C)")
    return _Modulate.apply(x, s, t, r, alpha, s.stride(0))


def attention_map(q, k, heads, scaling, average=True):
    """The attention weights of an MHA call with need_weights=True (multihead_attention.py:107-118):
    softmax(q_h k_h^T * scaling) over the keys, averaged over heads -> (B, N, S), else (B, H, N, S). A diagnostic
    output (the flash kernels never materialise it): returned without a gradient."""
    q, k = q.detach().float().contiguous(), k.detach().float().contiguous()
    B, N, E = q.shape
    S = k.shape[1]
    out = torch.empty((B, N, S) if average else (B, heads, N, S), dtype=torch.float32, device=q.device)
    _lib.check(_lib.lib().sdmi_attn_map(q.data_ptr(), E, k.data_ptr(), E, B, heads, N, S, E // heads, float(scaling),
                                        1 if average else 0, out.data_ptr(), K._stream()), "sdmi_attn_map")
    return out


# ---- dispatch -----------------------------------------------------------------------------------------------------
def call(mod, x, *rest):
    """Run leaf (or Sequential of leaves) `mod` on x: exact torch types on the HIP per-op path, anything else
    (a swapped layer) through its own forward."""
    t = type(mod)
    if t is nn.Sequential:
        mods = list(mod)
        i = 0
        while i < len(mods):
            if type(mods[i]) is nn.GroupNorm and i + 1 < len(mods) and type(mods[i + 1]) is nn.SiLU:
                x = group_norm(mods[i], x, silu=True)  # GroupNorm + SiLU in one kernel (blocks.py:45-55)
                i += 2
                continue
            x = call(mods[i], x)
            i += 1
        return x
    if t is nn.Conv2d:
        return conv2d(mod, x)
    if t is nn.ConvTranspose2d:
        return conv_transpose2d(mod, x)
    if t is nn.Linear:
        return linear(mod, x)
    if t is nn.GroupNorm:
        return group_norm(mod, x)
    if t is nn.SiLU:
        return _SiLU.apply(x)
    if t is nn.ReLU:
        return _ReLU.apply(x)
    if t is nn.LayerNorm:
        return layer_norm(mod, x)
    if t is nn.Identity or (t is nn.Dropout and not mod.training):
        return x
    if t is nn.MultiheadAttention:
        return multihead_attention(mod, x, *rest)
    return mod(x, *rest)


# exact torch types the fused whole-network engines implement; any other leaf type sends a model down this path
ENGINE_LEAVES = (nn.Conv2d, nn.ConvTranspose2d, nn.Linear, nn.GroupNorm, nn.SiLU, nn.ReLU, nn.Identity, nn.Dropout,
                 nn.MultiheadAttention, nn.Embedding, nn.LayerNorm, nn.Sequential, nn.ModuleList)


def engine_ok(model, containers=()):
    """True while every submodule is an exact engine leaf type or one of the model's own container classes
    (nn.MultiheadAttention's out_proj is torch's NonDynamicallyQuantizableLinear: part of the exact MHA)."""
    allowed = set(ENGINE_LEAVES) | set(containers) | {nn.modules.linear.NonDynamicallyQuantizableLinear}

    def ok(m):
        if type(m) not in allowed:
            return False
        # the engines apply no dropout: an active one (p > 0 in training mode; CustomMultiheadAttention builds
        # nn.Dropout(dropout), multihead_attention.py) takes the leaf path, which runs it
        if type(m) is nn.Dropout and m.training and m.p > 0:
            return False
        if type(m) is nn.MultiheadAttention and m.training and m.dropout > 0:
            return False
        return True
    return all(ok(m) for m in model.modules())


def time_embedding(t, B, dim, device):
    """get_time_embedding(t, dim) (blocks.py:5-24) as fp32 (B, dim) from the sdmi_time_embedding kernel."""
    tt = torch.as_tensor(t, device=device).long().reshape(-1).contiguous()
    out = torch.empty(B, dim, dtype=torch.float32, device=device)
    scratch = torch.empty(B, dim, dtype=torch.bfloat16, device=device)
    _lib.check(_lib.lib().sdmi_time_embedding(tt.data_ptr(), 0 if tt.numel() == 1 else 1, B, dim, scratch.data_ptr(),
                                              dim, out.data_ptr(), K._stream()), "sdmi_time_embedding")
    return out
