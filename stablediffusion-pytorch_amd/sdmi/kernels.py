"""Thin tensor-level wrappers over the C ABI (include/sdmi.h).

Every function here validates shapes on the host, then enqueues exactly the HIP kernels of
libsdmi.so on torch's current stream. Tensors are NHWC bf16 activations (2-D views [pixels, C]
with a row stride) and fp32 parameters/statistics.
"""
import ctypes

import torch

from . import _lib
from ._lib import GemmDesc, ConvGeom, check


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _log2(v):
    l = v.bit_length() - 1
    if (1 << l) != v:
        raise ValueError(f"spatial size {v} must be a power of two")
    return l


def gemm(m, n, k, a, a_mode, lda, b, b_mode, ldb, c, ldc, *, geom=None, bias=None, rowbias=None,
         rb_ld=0, rb_shift=0, resid=None, ldr=0, alpha=1.0, act=0, remap=None, perm=None):
    """C[m][n] = epi(sum_k A[m][k] B[k][n]).  a/b/c/resid/rowbias are tensors (pointer = data_ptr,
    offsets already applied by slicing); see include/sdmi.h for the operand modes."""
    L = _lib.lib()
    d = GemmDesc()
    d.m, d.n, d.k = m, n, k
    d.a_mode, d.b_mode = a_mode, b_mode
    d.a, d.lda = a.data_ptr(), lda
    d.b, d.ldb = b.data_ptr(), ldb
    if geom is not None:
        for f, v in geom.items():
            setattr(d.geom, f, v)
    d.c, d.ldc = c.data_ptr(), ldc
    d.c_f32 = 1 if c.dtype == torch.float32 else 0
    d.bias = bias.data_ptr() if bias is not None else None
    if rowbias is not None:
        d.rowbias, d.rb_ld, d.rb_shift = rowbias.data_ptr(), rb_ld, rb_shift
    if resid is not None:
        d.resid, d.ldr = resid.data_ptr(), ldr
    d.alpha = alpha
    d.act = act
    if remap is not None:
        (d.r_gh_log2, d.r_gw_log2, d.r_oh, d.r_ow, d.r_sy, d.r_sx, d.r_oy, d.r_ox) = remap
        d.remap = 1
    if perm is not None:
        d.perm = 1
        d.p_cin, d.p_taps = perm
    splits = ctypes.c_int(1)
    ws_bytes = ctypes.c_size_t(0)
    check(L.sdmi_gemm_plan(ctypes.byref(d), ctypes.byref(splits), ctypes.byref(ws_bytes)), "sdmi_gemm_plan")
    ws = None
    if ws_bytes.value:
        ws = torch.empty(ws_bytes.value // 4, dtype=torch.float32, device=c.device)
    check(L.sdmi_gemm(ctypes.byref(d), ws.data_ptr() if ws is not None else None, ws_bytes.value, _stream()),
          "sdmi_gemm")
    return c


# ------------------------------------------------------------------------------------------------
# convolution in NHWC as implicit GEMM
# ------------------------------------------------------------------------------------------------

def conv_geom(ih, iw, cin, ldx, kh, kw, oh, ow, sy, sx, oy0, ox0):
    return dict(ih=ih, iw=iw, cin=cin, ldx=ldx, kh=kh, kw=kw, oh_log2=_log2(oh), ow_log2=_log2(ow),
                sy=sy, sx=sx, oy0=oy0, ox0=ox0)


def conv_fwd(x, B, H, W, cin, ldx, wpk, cout, kh, kw, stride, pad, out, ldo, *, bias=None, rowbias=None,
             resid=None, ldr=0, act=0):
    """y[b,oy,ox,co] = sum_{ty,tx,ci} x[b, oy*s+ty-pad, ox*s+tx-pad, ci] * wpk[co, (ty*kw+tx)*cin + ci].
    x: NHWC bf16 buffer (row stride ldx), wpk: bf16 [cout][kh*kw*cin]."""
    OH = (H + 2 * pad - kh) // stride + 1
    OW = (W + 2 * pad - kw) // stride + 1
    g = conv_geom(H, W, cin, ldx, kh, kw, OH, OW, stride, stride, -pad, -pad)
    rb_shift = _log2(OH * OW)
    return gemm(B * OH * OW, cout, kh * kw * cin, x, _lib.A_CONV, 0, wpk, _lib.B_NK, kh * kw * cin, out, ldo,
                geom=g, bias=bias, rowbias=rowbias, rb_ld=cout if rowbias is not None else 0, rb_shift=rb_shift,
                resid=resid, ldr=ldr, act=act)


def conv_wgrad(dy, ldy, x, B, H, W, cin, ldx, cout, kh, kw, stride, pad, out, OH, OW, *, perm=True):
    """dW[co][(ty,tx,ci)] = sum_pixels dy[p, co] * x[gather(p, ty, tx), ci]; written fp32 in torch
    layout (co, ci, kh, kw) when perm."""
    g = conv_geom(H, W, cin, ldx, kh, kw, OH, OW, stride, stride, -pad, -pad)
    return gemm(cout, kh * kw * cin, B * OH * OW, dy, _lib.A_COLMAJOR, ldy, x, _lib.B_KN_CONV, 0, out,
                kh * kw * cin, geom=g, perm=(cin, kh * kw) if perm else None)


# stride-2, 4x4, pad-1 transposed convolution as four 2x2 sub-pixel convolutions.
# phase ph uses taps kh = 3 - ph - 2a (a = 0, 1) at input rows iy = oy + a + (ph - 1).
def phase_taps(ph):
    return [3 - ph - 2 * a for a in range(2)]


def convT_fwd_phases(x, B, H, W, cin, ldx, wph, cout, out, ldo, *, bias=None, resid=None, ldr=0):
    """Transposed conv k4 s2 p1: x (B,H,W,cin) -> out (B,2H,2W,cout).  wph: list of 4 packed bf16
    weights [cout][2*2*cin], phase index = ph*2 + pw."""
    for ph in range(2):
        for pw in range(2):
            g = conv_geom(H, W, cin, ldx, 2, 2, H, W, 1, 1, ph - 1, pw - 1)
            remap = (_log2(H), _log2(W), 2 * H, 2 * W, 2, 2, ph, pw)
            gemm(B * H * W, cout, 4 * cin, x, _lib.A_CONV, 0, wph[ph * 2 + pw], _lib.B_NK, 4 * cin, out, ldo,
                 geom=g, bias=bias, resid=resid, ldr=ldr, remap=remap)
    return out
