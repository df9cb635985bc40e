"""Thin tensor-level wrappers over the C ABI (include/sdmi.h).

Every function here validates shapes on the host, then enqueues exactly the HIP kernels of
libsdmi.so on torch's current stream. Tensors are NHWC bf16 activations (2-D views [pixels, C]
with a row stride) and fp32 parameters/statistics.
"""
import ctypes
import json
import os

import torch

from . import _lib
from ._lib import GemmDesc, ConvGeom, check


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


# optional per-launch timing hook (bench.py): list of (tag, flops, start_event, end_event, info)
PROFILE = None
# optional GEMM call log (scripts/plan_profile.py): list of (m, n, k, a_mode, b_mode, splits, tile_n, phase, kernel info)
GEMM_LOG = None
# optional descriptor capture (scripts/tune_gemm.py): copies of every GemmDesc issued while set (operands stay valid as
# long as the memory they point into does, e.g. a StepPlan's private pool)
GEMM_CAPTURE = None
PHASE = ""  # label prefixed to profiled launches ("fwd" / "bwd" / "wg" ...; set by the engines)
# phases whose GEMMs may take the 192-column tile (measured per phase: faster in fwd / bwd; in the weight-gradient
# phase its 80 KiB of LDS per workgroup crowds out the concurrent streams and the step ran 0.4 ms slower)
# elsewhere the 128-column tile is requested
TILE192_PHASES = {"fwd", "bwd"}

# measured split-K slice counts (or [splits, mainloop variant]) per GEMM shape (scripts/tune_gemm.py ->
# sdmi/tuned_gemm.json); None = not loaded
TUNED = None
_TUNED_PATH = os.environ.get("SDMI_TUNED_GEMM") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "tuned_gemm.json")


def gemm_key(d):
    """Shape key of a GemmDesc for the tuned split table."""
    g = d.geom
    return (f"a{d.a_mode}b{d.b_mode} m{d.m} n{d.n} k{d.k} g{g.kh}x{g.kw}s{g.sy} i{g.ih}c{g.cin} "
            f"x{int(bool(d.a2))}p{d.perm}")


def _tuned():
    global TUNED
    if TUNED is None:
        if os.environ.get("SDMI_TUNED_GEMM") and not os.path.exists(_TUNED_PATH):
            # an explicit table that is not there must not silently become the split heuristic
            raise FileNotFoundError(f"SDMI_TUNED_GEMM={_TUNED_PATH}: no such file")
        TUNED = json.load(open(_TUNED_PATH)) if os.path.exists(_TUNED_PATH) else {}
    return TUNED


class _Prof:
    """Context manager recording HIP events around a launch group when PROFILE is enabled."""

    def __init__(self, tag, flops, info=""):
        self.tag, self.flops, self.info = tag, flops, info

    def __enter__(self):
        if PROFILE is not None:
            self.e0 = torch.cuda.Event(enable_timing=True)
            self.e1 = torch.cuda.Event(enable_timing=True)
            self.e0.record()
        return self

    def __exit__(self, *a):
        if PROFILE is not None:
            self.e1.record()
            PROFILE.append((self.tag, self.flops, self.e0, self.e1, f"[{PHASE}] {self.info}" if PHASE else self.info))


# running total of the GEMM FLOPs issued (the UNet engine balances its weight-gradient side streams by it)
FLOPS_ISSUED = 0.0


def algo_bytes(d):
    """Algorithmic HBM bytes of one GEMM launch: every operand's UNIQUE bytes at its dtype, read or written once (an
    implicit-GEMM conv's im2col operand counts the activation it gathers from, not the k x taps expansion), plus the
    fused epilogue's addend / mask / second-source reads. The roofline's traffic / algorithmic ratio then shows what a
    kernel re-reads beyond that (split-K slabs, halo and cross-tile re-reads that miss L2)."""
    def conv_src(g, pixels):
        return (pixels // max(1, g.oh * g.ow)) * g.ih * g.iw * g.cin * 2
    m, n, k = d.m, d.n, d.k
    if d.a_mode == _lib.A_CONV:
        ka = d.k_split if d.a2 else k
        a = conv_src(d.geom, m) if ka else 0
        a += m * (k - d.k_split) * 2 if d.a2 else 0
    else:
        a = m * k * 2
    b = conv_src(d.geom, k) if d.b_mode == _lib.B_KN_CONV else n * k * 2
    ms, ns = (d.m_store or m), (d.n_store or n)
    out = ms * ns * (4 if d.c_f32 else 2)
    extra = (ms * ns * 2 if d.resid else 0) + (ms * ns * 2 if d.aux else 0)
    return a + b + out + extra


def gemm(m, n, k, a, a_mode, lda, b, b_mode, ldb, c, ldc, *, geom=None, bias=None, rowbias=None,
         rb_ld=0, rb_div=0, resid=None, ldr=0, alpha=1.0, act=0, remap=None, perm=None, m_store=0, n_store=0,
         a2=None, lda2=0, k_split=0, bias2=None, rb_mod=0, aux=None, ld_aux=0, sum_out=None, sum_out2=None,
         gsum=None, sum_group=0, gn=None):
    """C[m][n] = epi(sum_k A[m][k] B[k][n]).  a/b/c/resid/rowbias are tensors (pointer = data_ptr,
    offsets already applied by slicing); see include/sdmi.h for the operand modes.
    gn (gn_request): C is the data gradient of a [SiLU(]GroupNorm(x)[)] output; the launch also writes the
    GroupNorm-backward segment statistics (sdmi_gemm_desc::gn_part) into gn["part"] (rows per segment gn["rb"])."""
    global FLOPS_ISSUED
    FLOPS_ISSUED += 2.0 * m * n * k
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
        d.rowbias, d.rb_ld, d.rb_div = rowbias.data_ptr(), rb_ld, rb_div
    if resid is not None:
        d.resid, d.ldr = resid.data_ptr(), ldr
    d.alpha = alpha
    d.act = act
    if remap is not None:
        (d.r_gh, d.r_gw, d.r_oh, d.r_ow, d.r_sy, d.r_sx, d.r_oy, d.r_ox) = remap
        d.remap = 1
    if perm is not None:
        d.perm = perm[3] if len(perm) > 3 else 1
        d.p_cin, d.p_taps = perm[0], perm[1]
        d.p_cvalid = perm[2] if len(perm) > 2 else 0
    d.m_store, d.n_store = m_store, n_store
    if a2 is not None:
        d.a2, d.lda2, d.k_split = a2.data_ptr(), lda2, k_split
    d.bias2 = bias2.data_ptr() if bias2 is not None else None
    d.rb_mod = rb_mod
    if aux is not None:
        d.aux, d.ld_aux = aux.data_ptr(), ld_aux or ld_of(aux)
    if sum_out is not None or sum_out2 is not None or gsum is not None:  # reductions of A (col-major A only)
        d.sum_out = _p(sum_out)
        d.sum_out2 = _p(sum_out2)
        if gsum is not None:
            d.gsum_out, d.gsum_ld, d.sum_group = gsum.data_ptr(), ld_of(gsum), sum_group
    d.tile_n_hint = 0 if (not PHASE or PHASE in TILE192_PHASES) else 128
    if gn is not None:
        d.gn_x, d.gn_ldx = gn["x"].data_ptr(), ld_of(gn["x"])
        d.gn_tab = gn["tab"].data_ptr()
        d.gn_P, d.gn_silu = gn["P"], 1 if gn.get("silu") else 0
        d.gn_rb = gn_rb(gn["P"], 64)
        d.gn_part = 8  # validated by the plan; the real buffer once the split count (and so the segment) is known
    tuned = _tuned()
    if tuned:
        e = tuned.get(gemm_key(d), 0)  # splits, or [splits, mainloop variant]
        if isinstance(e, list):
            d.splits_hint, d.variant_hint = e[0], e[1]
        else:
            d.splits_hint = e
    splits = ctypes.c_int(1)
    ws_bytes = ctypes.c_size_t(0)
    check(L.sdmi_gemm_plan(ctypes.byref(d), ctypes.byref(splits), ctypes.byref(ws_bytes)), "sdmi_gemm_plan")
    if gn is not None:
        rb = gn_rb(gn["P"], 64 if splits.value == 1 else 16)
        part = torch.empty(m // rb * n * 2, dtype=torch.float32, device=c.device)
        d.gn_rb, d.gn_part = rb, part.data_ptr()
        gn["part"], gn["rb"] = part, rb
    if GEMM_CAPTURE is not None:
        GEMM_CAPTURE.append(GemmDesc.from_buffer_copy(d))
    ws = None
    if ws_bytes.value:
        ws = torch.empty(ws_bytes.value // 4, dtype=torch.float32, device=c.device)
    info = ""
    if GEMM_LOG is not None:
        var, tn = ctypes.c_int(0), ctypes.c_int(0)
        check(L.sdmi_gemm_kernel_info(ctypes.byref(d), ctypes.byref(var), ctypes.byref(tn)), "sdmi_gemm_kernel_info")
        GEMM_LOG.append(dict(m=m, n=n, k=k, a=a_mode, b=b_mode, splits=splits.value, tile_n=tn.value, variant=var.value,
                             phase=PHASE, conv=geom is not None and a_mode == _lib.A_CONV and (geom or {}).get("kh", 1),
                             flops=2.0 * m * n * k))
    if PROFILE is not None:  # attribute the launch to its kernel instantiation (roofline / profiles)
        var, tn = ctypes.c_int(0), ctypes.c_int(0)
        check(L.sdmi_gemm_kernel_info(ctypes.byref(d), ctypes.byref(var), ctypes.byref(tn)), "sdmi_gemm_kernel_info")
        info = f" variant={var.value} tile_n={tn.value}"
        info += f" bytes={algo_bytes(d)}"
    with _Prof(f"gemm_a{a_mode}b{b_mode}", 2.0 * m * n * k, f"M={m} N={n} K={k} splits={splits.value}{info}"):
        check(L.sdmi_gemm(ctypes.byref(d), ws.data_ptr() if ws is not None else None, ws_bytes.value, _stream()),
              "sdmi_gemm")
    return c


# ------------------------------------------------------------------------------------------------
# convolution in NHWC as implicit GEMM
# ------------------------------------------------------------------------------------------------

def conv_geom(ih, iw, cin, ldx, kh, kw, oh, ow, sy, sx, oy0, ox0):
    if oh <= 0 or ow <= 0:
        raise ValueError(f"empty convolution output grid {oh} x {ow}")
    return dict(ih=ih, iw=iw, cin=cin, ldx=ldx, kh=kh, kw=kw, oh=oh, ow=ow,
                sy=sy, sx=sx, oy0=oy0, ox0=ox0)


def conv_fwd(x, B, H, W, cin, ldx, wpk, cout, kh, kw, stride, pad, out, ldo, *, bias=None, rowbias=None,
             rb_ld=0, resid=None, ldr=0, act=0, n_store=0, x2=None, cin2=0, bias2=None, ldw=0, gn=None):
    """y[b,oy,ox,co] = sum_{ty,tx,ci} x[b, oy*s+ty-pad, ox*s+tx-pad, ci] * wpk[co, (ty*kw+tx)*cin + ci].
    x: NHWC bf16 buffer (row stride ldx), wpk: bf16 [cout][kh*kw*cin]."""
    OH = (H + 2 * pad - kh) // stride + 1
    OW = (W + 2 * pad - kw) // stride + 1
    g = conv_geom(H, W, cin, ldx, kh, kw, OH, OW, stride, stride, -pad, -pad)
    K1 = kh * kw * cin
    if x2 is not None:  # fused 1x1 conv of x2 (same pixel grid) by K-concatenation: wpk = [W | W2]
        assert stride == 1 and OH == H and OW == W
    return gemm(B * OH * OW, cout, K1 + cin2, x, _lib.A_CONV, 0, wpk, _lib.B_NK, ldw or (K1 + cin2), out, ldo,
                geom=g, bias=bias, rowbias=rowbias, rb_ld=(rb_ld or cout) if rowbias is not None else 0,
                rb_div=OH * OW, resid=resid, ldr=ldr, act=act, n_store=n_store,
                a2=x2, lda2=ld_of(x2) if x2 is not None else 0, k_split=K1, bias2=bias2, gn=gn)


def conv_wgrad(dy, ldy, x, B, H, W, cin, ldx, cout, kh, kw, stride, pad, out, OH, OW, *, perm=True, cvalid=0,
               m_store=0, bias_grad=None, bias_grad2=None, group_sums=None):
    """dW[co][(ty,tx,ci)] = sum_pixels dy[p, co] * x[gather(p, ty, tx), ci]; written fp32 in torch
    layout (co, ci, kh, kw) when perm is True (only ci < cvalid, co < m_store when given); perm may also be
    an explicit (p_cin, p_taps, p_cvalid, mode) tuple (mode 2: tap-major (co, kh, kw, ci) Linear layout).
    In the same launch: bias_grad[co] (and bias_grad2) = sum_pixels dy[p, co], group_sums[b][co] (bf16 2-D view) =
    per-sample sums -- the column-sum passes of the conv bias and time-embedding gradients."""
    g = conv_geom(H, W, cin, ldx, kh, kw, OH, OW, stride, stride, -pad, -pad)
    cv = cvalid or cin
    if perm is True:
        perm = (cin, kh * kw, cv)
    elif isinstance(perm, tuple):
        cv = perm[2]
    return gemm(cout, kh * kw * cin, B * OH * OW, dy, _lib.A_COLMAJOR, ldy, x, _lib.B_KN_CONV, 0, out,
                kh * kw * cv, geom=g, perm=perm or None, m_store=m_store, sum_out=bias_grad, sum_out2=bias_grad2,
                gsum=group_sums, sum_group=OH * OW)


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
            remap = (H, W, 2 * H, 2 * W, 2, 2, ph, pw)
            gemm(B * H * W, cout, 4 * cin, x, _lib.A_CONV, 0, wph[ph * 2 + pw], _lib.B_NK, 4 * cin, out, ldo,
                 geom=g, bias=bias, resid=resid, ldr=ldr, remap=remap)
    return out


# ------------------------------------------------------------------------------------------------
# tensor helpers
# ------------------------------------------------------------------------------------------------
def ld_of(t):
    """row stride (elements) of a 2-D [rows, C] view with unit column stride."""
    assert t.dim() == 2 and t.stride(1) == 1, "activation views must be 2-D with unit column stride"
    return t.stride(0)


def _p(t):
    return t.data_ptr() if t is not None else None


def linear(x, w, out, *, bias=None, resid=None, act=0, alpha=1.0, n_store=0, rowbias=None, rb_mod=0, gn=None):
    """out[m][n] = act(alpha * x[m] . w[n] + bias[n] + rowbias[m % rb_mod][n] + resid[m][n]);
    x [M,K] bf16 view, w [N,K] bf16 (act: 0 none, 1 SiLU, 2 ReLU)."""
    M, K = x.shape
    N = w.shape[0]
    return gemm(M, N, K, x, _lib.A_ROWMAJOR, ld_of(x), w, _lib.B_NK, ld_of(w), out, ld_of(out), bias=bias,
                resid=resid, ldr=ld_of(resid) if resid is not None else 0, act=act, alpha=alpha, n_store=n_store,
                rowbias=rowbias, rb_ld=ld_of(rowbias) if rowbias is not None else 0, rb_mod=rb_mod, gn=gn)


def linear_dgrad(dy, w, out, *, resid=None, relu_of=None, gn=None):
    """out[m][k] = sum_n dy[m][n] w[n][k] (+ resid), times (relu_of[m][k] > 0) when relu_of (the saved ReLU
    output) is given;  w [N,K] bf16 used as B[k=n][n=k] (row-major)."""
    M, N = dy.shape
    K = w.shape[1]
    return gemm(M, K, N, dy, _lib.A_ROWMAJOR, ld_of(dy), w, _lib.B_KN, w.stride(0), out, ld_of(out), resid=resid,
                ldr=ld_of(resid) if resid is not None else 0, act=3 if relu_of is not None else 0, aux=relu_of, gn=gn)


def linear_dgrad_t(dy, wt, out, *, resid=None, relu_of=None, gn=None):
    """linear_dgrad from the transposed weight: out[m][k] = sum_n dy[m][n] wt[k][n] (+ resid, ReLU mask as
    linear_dgrad); wt [K,N] bf16 rows (B_NK), which takes the wider N tiles of the forward GEMM."""
    M, N = dy.shape
    K = wt.shape[0]
    return gemm(M, K, N, dy, _lib.A_ROWMAJOR, ld_of(dy), wt, _lib.B_NK, ld_of(wt), out, ld_of(out), resid=resid,
                ldr=ld_of(resid) if resid is not None else 0, act=3 if relu_of is not None else 0, aux=relu_of, gn=gn)


def linear_wgrad(dy, x, out, *, bias_grad=None, bias_grad2=None, group_sums=None, group=0, m_store=0):
    """out[n][k] = sum_m dy[m][n] x[m][k]  (fp32 weight gradient, out [N,K] contiguous rows); in the same launch
    bias_grad[n] (and bias_grad2) = sum_m dy[m][n] and group_sums[g][n] (bf16) = sums over rows [g*group, ...)."""
    M, N = dy.shape
    K = x.shape[1]
    return gemm(N, K, M, dy, _lib.A_COLMAJOR, ld_of(dy), x, _lib.B_KN, ld_of(x), out, out.stride(0),
                sum_out=bias_grad, sum_out2=bias_grad2, gsum=group_sums, sum_group=group, m_store=m_store)


# Mainloop of grouped weight-gradient launches: variant 3 (LDS-DMA ring, 3 stages of 32-deep k; variant 2 where bias
# reduction columns ride along). The tuned table holds single-problem entries, mostly the register-staged mainloop,
# which lost to the DMA ring once 6-8 problems share the grid. Same box: cond-UNet 13.36 / 13.30 -> 13.29 / 13.27 ms,
# DiT-12L 3.56 / 3.56 -> 3.53 / 3.52 ms.
GROUPED_VARIANT = int(os.environ.get("SDMI_GROUPED_VARIANT", "3"))  # diagnostic override (A/B of mainloops)


def linear_wgrad_grouped(items):
    """linear_wgrad of several same-shape problems in ONE launch (sdmi_gemm_grouped): items = [(dy, x, out,
    bias_grad or None)], all dy / x of one shape and row stride, all bias_grad present or all None. The split count is
    the single problem's tuned one shared out over the group."""
    global FLOPS_ISSUED
    G = len(items)
    if G == 1:
        dy, x, out, bg = items[0]
        linear_wgrad(dy, x, out, bias_grad=bg)
        return
    L = _lib.lib()
    descs = (GemmDesc * G)()
    M, N = items[0][0].shape
    K = items[0][1].shape[1]
    FLOPS_ISSUED += 2.0 * M * N * K * G
    for i, (dy, x, out, bg) in enumerate(items):
        d = descs[i]
        d.m, d.n, d.k = N, K, M
        d.a_mode, d.b_mode = _lib.A_COLMAJOR, _lib.B_KN
        d.a, d.lda = dy.data_ptr(), ld_of(dy)
        d.b, d.ldb = x.data_ptr(), ld_of(x)
        d.c, d.ldc, d.c_f32 = out.data_ptr(), out.stride(0), 1
        d.alpha = 1.0
        d.sum_out = _p(bg)
        d.tile_n_hint = 0 if (not PHASE or PHASE in TILE192_PHASES) else 128
    tuned = _tuned()
    if tuned:
        e = tuned.get(gemm_key(descs[0]), 0)
        for i in range(G):
            if isinstance(e, list):
                descs[i].splits_hint, descs[i].variant_hint = e[0], e[1]
            else:
                descs[i].splits_hint = e
    for i in range(G):  # the LDS-DMA mainloop (GROUPED_VARIANT), whatever the single problem's tuned entry
        descs[i].variant_hint = GROUPED_VARIANT
    splits = ctypes.c_int(1)
    ws_bytes = ctypes.c_size_t(0)
    check(L.sdmi_gemm_grouped_plan(descs, G, ctypes.byref(splits), ctypes.byref(ws_bytes)), "sdmi_gemm_grouped_plan")
    ws = torch.empty(ws_bytes.value // 4, dtype=torch.float32, device=items[0][2].device) if ws_bytes.value else None
    if GEMM_LOG is not None:
        var, tn = ctypes.c_int(0), ctypes.c_int(0)
        check(L.sdmi_gemm_kernel_info(ctypes.byref(descs[0]), ctypes.byref(var), ctypes.byref(tn)), "kernel_info")
        GEMM_LOG.append(dict(m=N, n=K, k=M, a=_lib.A_COLMAJOR, b=_lib.B_KN, splits=splits.value, tile_n=tn.value,
                             variant=var.value, phase=PHASE, conv=False, flops=2.0 * M * N * K * G, groups=G))
    info = ""
    if PROFILE is not None:
        var, tn = ctypes.c_int(0), ctypes.c_int(0)
        check(L.sdmi_gemm_kernel_info(ctypes.byref(descs[0]), ctypes.byref(var), ctypes.byref(tn)), "kernel_info")
        info = f" variant={var.value} tile_n={tn.value} bytes={sum(algo_bytes(x) for x in descs[:G])}"
    with _Prof(f"gemm_a{_lib.A_COLMAJOR}b{_lib.B_KN}", 2.0 * M * N * K * G,
               f"M={N} N={K} K={M} splits={splits.value} groups={G}{info}"):
        check(L.sdmi_gemm_grouped(descs, G, ws.data_ptr() if ws is not None else None, ws_bytes.value, _stream()),
              "sdmi_gemm_grouped")


def gn_stats(x, B, P, C, G, gamma, beta, eps=1e-5):
    """GroupNorm statistics -> per-(b,c) table {rstd*gamma, beta - mean*rstd*gamma, mean, rstd} fp32 [B*C*4]."""
    L = _lib.lib()
    ws = torch.empty(L.sdmi_chan_reduce_workspace(B, P, C) // 4, dtype=torch.float32, device=x.device)
    tab = torch.empty(B * C * 4, dtype=torch.float32, device=x.device)
    with _Prof("gn_stats", 0, f"B={B} P={P} C={C}"):
        check(L.sdmi_gn_stats(_p(x), ld_of(x), B, P, C, G, eps, _p(gamma), _p(beta), _p(ws), _p(tab), _stream()),
              "sdmi_gn_stats")
    return tab


def gn_fwd(x, B, P, C, G, gamma, beta, silu, out, eps=1e-5):
    """out = [SiLU](GroupNorm(x)); returns the forward table (as gn_stats) for the backward pass."""
    L = _lib.lib()
    ws = torch.empty(L.sdmi_chan_reduce_workspace(B, P, C) // 4, dtype=torch.float32, device=x.device)
    tab = torch.empty(B * C * 4, dtype=torch.float32, device=x.device)
    with _Prof("gn_fwd", 0, f"B={B} P={P} C={C}"):
        check(L.sdmi_gn_fwd(_p(x), ld_of(x), _p(out), ld_of(out), B, P, C, G, eps, _p(gamma), _p(beta),
                            1 if silu else 0, _p(ws), _p(tab), _stream()), "sdmi_gn_fwd")
    return tab


def gn_apply(x, tab, B, P, C, silu, out):
    with _Prof("gn_apply", 0, f"B={B} P={P} C={C}"):
        check(_lib.lib().sdmi_gn_apply(_p(x), ld_of(x), _p(out), ld_of(out), _p(tab), B, P, C, 1 if silu else 0,
                                       _stream()), "sdmi_gn_apply")
    return out


def gn_rb(P, cap):
    """rows per GroupNorm-backward statistics segment: the largest of 64 / 32 / 16 (<= cap) dividing P, else 0"""
    for rb in (64, 32, 16):
        if rb <= cap and P % rb == 0:
            return rb
    return 0


def gn_request(x, tab, P, C, silu):
    """GroupNorm-backward statistics request for the GEMM producing the GroupNorm output gradient (gemm(gn=...)), or
    None where the fused path does not apply (P % 16 != 0: e.g. MNIST's 7 x 7 level; C % 8 != 0)."""
    if P % 16 or C % 8 or ld_of(x) % 8:
        return None
    return dict(x=x, tab=tab, P=P, silu=silu)


def gn_bwd(x, dy, dx, tab, gamma, B, P, C, G, silu, dgamma, dbeta, addend=None, gn=None, defer=None):
    """GroupNorm(+SiLU) backward; with gn (the request whose GEMM produced dy) from its segment statistics in one
    streaming launch (sdmi_gn_bwd_part), else the self-contained sdmi_gn_bwd. defer (a list): dgamma / dbeta are not
    summed by this launch -- its per-(batch row, channel) sums go to a rows buffer and (rows, B, C, dgamma, dbeta) is
    appended to defer for gn_rows_sum (the caller issues it off the data-gradient chain)."""
    L = _lib.lib()
    ws = torch.empty(L.sdmi_chan_reduce_workspace(B, P, C) // 4, dtype=torch.float32, device=x.device)
    rows = torch.empty(B * C * 2, dtype=torch.float32, device=x.device) if defer is not None else None
    add = (_p(addend), ld_of(addend) if addend is not None else 0)
    if gn is not None:
        assert gn.get("part") is not None, "the producing GEMM did not run with this GroupNorm request"
        with _Prof("gn_bwd", 0, f"B={B} P={P} C={C} part"):
            if rows is None:
                check(L.sdmi_gn_bwd_part(_p(x), ld_of(x), _p(dy), ld_of(dy), _p(dx), ld_of(dx), _p(tab), _p(gamma), B, P,
                                         C, G, 1 if silu else 0, _p(gn["part"]), gn["rb"], _p(ws), _p(dgamma),
                                         _p(dbeta), *add, _stream()), "sdmi_gn_bwd_part")
            else:
                check(L.sdmi_gn_bwd_part_rows(_p(x), ld_of(x), _p(dy), ld_of(dy), _p(dx), ld_of(dx), _p(tab), _p(gamma),
                                              B, P, C, G, 1 if silu else 0, _p(gn["part"]), gn["rb"], _p(ws),
                                              _p(rows), *add, _stream()), "sdmi_gn_bwd_part_rows")
    else:
        tab2 = torch.empty(B * C * 4, dtype=torch.float32, device=x.device)
        with _Prof("gn_bwd", 0, f"B={B} P={P} C={C}"):
            if rows is None:
                check(L.sdmi_gn_bwd(_p(x), ld_of(x), _p(dy), ld_of(dy), _p(dx), ld_of(dx), _p(tab), _p(gamma), B, P, C,
                                    G, 1 if silu else 0, _p(ws), _p(tab2), _p(dgamma), _p(dbeta), *add, _stream()),
                      "sdmi_gn_bwd")
            else:
                check(L.sdmi_gn_bwd_rows(_p(x), ld_of(x), _p(dy), ld_of(dy), _p(dx), ld_of(dx), _p(tab), _p(gamma), B,
                                         P, C, G, 1 if silu else 0, _p(ws), _p(tab2), _p(rows), *add, _stream()),
                      "sdmi_gn_bwd_rows")
    if rows is not None:
        defer.append((rows, B, C, dgamma, dbeta))
    return dx


def gn_rows_sum(rows, B, C, dgamma, dbeta):
    """dgamma / dbeta from a deferred GroupNorm backward's rows buffer (gn_bwd(defer=...))."""
    with _Prof("gn_rows_sum", 0, f"B={B} C={C}"):
        check(_lib.lib().sdmi_gn_rows_sum(_p(rows), B, C, _p(dgamma), _p(dbeta), _stream()), "sdmi_gn_rows_sum")


def gn_rows_sum_grouped(jobs):
    """Several deferred GroupNorm sums [(rows, B, C, dgamma, dbeta), ...] in one launch (bitwise gn_rows_sum each)."""
    import ctypes
    for i in range(0, len(jobs), _lib.GN_ROWS_GROUP_MAX):
        part = jobs[i:i + _lib.GN_ROWS_GROUP_MAX]
        arr = (_lib.GnRowsJob * len(part))(*[_lib.GnRowsJob(_p(r), _p(dg), _p(db), B, C) for r, B, C, dg, db in part])
        with _Prof("gn_rows_sum", 0, f"grouped n={len(part)}"):
            check(_lib.lib().sdmi_gn_rows_sum_grouped(ctypes.cast(arr, ctypes.c_void_p), len(part), _stream()),
                  "sdmi_gn_rows_sum_grouped")


def chan_sum(dy, B, P, C, *, per_bc=None, per_c=None, per_c2=None, c_store=0):
    """per-(b,c) sums over pixels -> per_bc (bf16 2-D view [B, ld]) and per-channel sums (fp32)."""
    L = _lib.lib()
    ws = torch.empty(L.sdmi_chan_reduce_workspace(B, P, C) // 4, dtype=torch.float32, device=dy.device)
    with _Prof("chan_sum", 0, f"B={B} P={P} C={C}"):
        check(L.sdmi_chan_sum(_p(dy), ld_of(dy), B, P, C, _p(ws), _p(per_bc), ld_of(per_bc) if per_bc is not None else 0,
                          _p(per_c), _p(per_c2), c_store, _stream()), "sdmi_chan_sum")


def attn_fwd(q, k, v, out, B, H, N, S, d):
    lse = torch.empty(B * H * N, dtype=torch.float32, device=q.device)
    with _Prof("attn_fwd", 4.0 * B * H * N * S * d, f"B={B} H={H} N={N} S={S} d={d}"):
      check(_lib.lib().sdmi_attn_fwd(_p(q), ld_of(q), _p(k), ld_of(k), _p(v), ld_of(v), _p(out), ld_of(out), _p(lse),
                                   B, H, N, S, d, _stream()), "sdmi_attn_fwd")
    return lse


# Attention backward: the fused one-pass kernel (attn_bwd_fused_kernel) where all keys fit one 128-key block and
# there are >= 512 queries -- the 32x32 cross-attention over the 77 text tokens, dQ stored directly: 59.8 -> 50.6 us
# at d = 16, 71.3 -> 68.7 us at d = 24 (B = 32, N = 1024). Otherwise the dQ pass + dK/dV pass: at S = 1024 the
# fused kernel's cross-block dQ partials made it 1.5-4x slower (296 -> 490 us at d = 16, 322 -> 1347 us at d = 24),
# and at N = S = 64 / 16 its single query tile per workgroup lost 1-2 us. SDMI_ATTN_FUSED=0 / 1 forces either path.
ATTN_FUSED = os.environ.get("SDMI_ATTN_FUSED", "auto")


def attn_bwd(q, k, v, o, dout, lse, dq, dk, dv, B, H, N, S, d, fused=None):
    L = _lib.lib()
    delta = torch.empty(B * H * N, dtype=torch.float32, device=q.device)
    if fused is None:
        fused = (S <= 128 and N >= 512) if ATTN_FUSED == "auto" else ATTN_FUSED != "0"
    with _Prof("attn_bwd", 10.0 * B * H * N * S * d, f"B={B} H={H} N={N} S={S} d={d}"):
        if fused:
            nws = L.sdmi_attn_bwd_workspace(B, H, N, S, d)
            ws = torch.empty(max(nws // 4, 1), dtype=torch.float32, device=q.device)
            check(L.sdmi_attn_bwd_fused(_p(q), ld_of(q), _p(k), ld_of(k), _p(v), ld_of(v), _p(o), ld_of(o), _p(dout),
                                        ld_of(dout), _p(lse), _p(delta), _p(ws), nws, _p(dq), ld_of(dq), _p(dk),
                                        ld_of(dk), _p(dv), ld_of(dv), B, H, N, S, d, _stream()), "sdmi_attn_bwd_fused")
        else:
            check(L.sdmi_attn_bwd(_p(q), ld_of(q), _p(k), ld_of(k), _p(v), ld_of(v), _p(o), ld_of(o), _p(dout),
                                  ld_of(dout), _p(lse), _p(delta), _p(dq), ld_of(dq), _p(dk), ld_of(dk), _p(dv),
                                  ld_of(dv), B, H, N, S, d, _stream()), "sdmi_attn_bwd")


def conv_dgrad_phases(dy, B, H, W, cout, ldy, wph, cin, out, ldo, *, resid=None, ldr=0):
    """Gradient of a k4 s2 p1 convolution (input H x W -> output H/2 x W/2) w.r.t. its input, as four
    2x2 sub-pixel convolutions over dy (B, H/2, W/2, cout). wph[ph*2+pw]: bf16 [cin][2*2*cout]."""
    h, w = H // 2, W // 2
    for ph in range(2):
        for pw in range(2):
            g = conv_geom(h, w, cout, ldy, 2, 2, h, w, 1, 1, ph - 1, pw - 1)
            remap = (h, w, H, W, 2, 2, ph, pw)
            gemm(B * h * w, cin, 4 * cout, dy, _lib.A_CONV, 0, wph[ph * 2 + pw], _lib.B_NK, 4 * cout, out, ldo,
                 geom=g, resid=resid, ldr=ldr, remap=remap)
    return out


def add_noise(x0, eps, t, sqrt_abar, sqrt_1m_abar, out):
    B = x0.shape[0]
    check(_lib.lib().sdmi_add_noise(_p(x0), _p(eps), _p(t), _p(sqrt_abar), _p(sqrt_1m_abar), B, x0.numel() // B,
                                    _p(out), _stream()), "sdmi_add_noise")
    return out


def mse(pred, ld, target, B, C, HW, gscale, grad, loss, gscale_dev=None):
    ws = torch.empty(_lib.lib().sdmi_mse_workspace() // 4, dtype=torch.float32, device=pred.device)
    check(_lib.lib().sdmi_mse(_p(pred), ld, _p(target), B, C, HW, gscale, _p(gscale_dev), _p(grad), _p(ws), _p(loss),
                              _stream()), "sdmi_mse")


def copy_slice(src, dst, accumulate=False):
    P, C = src.shape
    check(_lib.lib().sdmi_copy_slice(_p(src), ld_of(src), _p(dst), ld_of(dst), P, C, 1 if accumulate else 0,
                                     _stream()), "sdmi_copy_slice")


def is_class_map(mask):
    """A (B, MH, MW) uint8 class map (sdmi.latents mask shards) instead of the reference's (B, cmi, MH, MW) fp32
    one-hot (dataset/celeb_dataset.py:164-175)."""
    return mask is not None and mask.dtype == torch.uint8 and mask.dim() == 3


def prep_input(x, B, cx, H, W, mask, cmi, wcond, cmo, out, cpad, keep):
    """Network input staging (unet_cond_base.py:131-140 / transformer.py:180-188): x NCHW fp32 -> NHWC bf16 with
    the nearest-resized mask through the 1x1 cond conv; the mask is a one-hot fp32 tensor or a uint8 class map."""
    L = _lib.lib()
    if mask is None:
        _lib.check(L.sdmi_prep_input(_ptr(x), B, cx, H, W, None, 0, 1, 1, None, 0, _ptr(out), cpad, None, _stream()),
                   "sdmi_prep_input")
    elif is_class_map(mask):
        _lib.check(L.sdmi_prep_input_cmap(_ptr(x), B, cx, H, W, _ptr(mask), cmi, mask.shape[1], mask.shape[2],
                                          _ptr(wcond), cmo, _ptr(out), cpad, _p(keep), _stream()),
                   "sdmi_prep_input_cmap")
    else:
        _lib.check(L.sdmi_prep_input(_ptr(x), B, cx, H, W, _ptr(mask), cmi, mask.shape[2], mask.shape[3],
                                     _ptr(wcond), cmo, _ptr(out), cpad, _p(keep), _stream()), "sdmi_prep_input")


def cond_wgrad(dxin, ld, cx, B, H, W, mask, cmi, cmo, dw, keep):
    """Gradient of cond_conv_in.weight from the staged-input gradient (one-hot or class-map mask)."""
    L = _lib.lib()
    if is_class_map(mask):
        _lib.check(L.sdmi_cond_wgrad_cmap(_ptr(dxin), ld, cx, B, H, W, _ptr(mask), cmi, mask.shape[1],
                                          mask.shape[2], cmo, _ptr(dw), _p(keep), _stream()), "sdmi_cond_wgrad_cmap")
    else:
        _lib.check(L.sdmi_cond_wgrad(_ptr(dxin), ld, cx, B, H, W, _ptr(mask), cmi, mask.shape[2], mask.shape[3], cmo,
                                     _ptr(dw), _p(keep), _stream()), "sdmi_cond_wgrad")
