"""GPU numerics of the MFMA GEMM family (libsdmi.so sdmi_gemm) against torch fp32 references of
the same op on bf16-rounded operands.  Tolerance: bf16 output rounding (2^-8 relative) plus fp32
accumulation-order differences."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _k():
    from sdmi import kernels, _lib
    return kernels, _lib


def bf(t):
    return t.to(torch.bfloat16)


def close(out, ref, tol=1e-2):
    err = (out.float() - ref.float()).abs().max().item()
    scale = ref.float().abs().max().item() + 1e-6
    assert err <= tol * scale, f"max err {err} vs scale {scale}"


@pytest.mark.parametrize("M,N,K", [(300, 200, 136), (128, 128, 64), (17, 40, 8), (64, 768, 4608)])
def test_rowmajor_nk(M, N, K):
    k, L = _k()
    torch.manual_seed(0)
    a = bf(torch.randn(M, K, device="cuda"))
    w = bf(torch.randn(N, K, device="cuda"))
    bias = torch.randn(N, device="cuda")
    res = bf(torch.randn(M, N, device="cuda"))
    c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    k.gemm(M, N, K, a, L.A_ROWMAJOR, K, w, L.B_NK, K, c, N, bias=bias, resid=res, ldr=N)
    ref = a.float() @ w.float().t() + bias + res.float()
    close(c, ref)
    c32 = torch.empty(M, N, device="cuda")
    k.gemm(M, N, K, a, L.A_ROWMAJOR, K, w, L.B_NK, K, c32, N, act=1, alpha=0.5)
    close(c32, F.silu(0.5 * (a.float() @ w.float().t())), 2e-3)


@pytest.mark.parametrize("M,N,K", [(257, 136, 72), (2048, 512, 384)])
def test_rowmajor_kn(M, N, K):
    k, L = _k()
    torch.manual_seed(1)
    a = bf(torch.randn(M, K, device="cuda"))
    b = bf(torch.randn(K, N, device="cuda"))
    c = torch.empty(M, N, device="cuda")
    k.gemm(M, N, K, a, L.A_ROWMAJOR, K, b, L.B_KN, N, c, N)
    close(c, a.float() @ b.float(), 2e-3)


@pytest.mark.parametrize("M,N,K", [(136, 264, 200), (512, 512, 32768)])
def test_colmajor_kn(M, N, K):
    k, L = _k()
    torch.manual_seed(2)
    at = bf(torch.randn(K, M, device="cuda"))
    b = bf(torch.randn(K, N, device="cuda"))
    c = torch.empty(M, N, device="cuda")
    k.gemm(M, N, K, at, L.A_COLMAJOR, M, b, L.B_KN, N, c, N)
    close(c, at.float().t() @ b.float(), 2e-3)


@pytest.mark.parametrize("B,H,cin,cout,ks,stride,pad", [
    (2, 8, 16, 24, 3, 1, 1), (2, 16, 8, 32, 3, 1, 1), (3, 8, 64, 64, 4, 2, 1), (2, 4, 32, 16, 1, 1, 0),
    (4, 32, 128, 136, 3, 1, 1)])
def test_conv_fwd_and_wgrad(B, H, cin, cout, ks, stride, pad):
    k, L = _k()
    torch.manual_seed(3)
    x = bf(torch.randn(B, cin, H, H, device="cuda"))
    w = bf(torch.randn(cout, cin, ks, ks, device="cuda") * 0.1)
    ref = F.conv2d(x.float().cpu(), w.float().cpu(), stride=stride, padding=pad).cuda()  # host fp32 reference
    OH = ref.shape[-1]
    xn = x.permute(0, 2, 3, 1).contiguous()
    wpk = w.permute(0, 2, 3, 1).contiguous()
    out = torch.empty(B, OH, OH, cout, device="cuda", dtype=torch.bfloat16)
    rowbias = bf(torch.randn(B, cout, device="cuda"))
    k.conv_fwd(xn, B, H, H, cin, cin, wpk, cout, ks, ks, stride, pad, out, cout, rowbias=rowbias)
    close(out.permute(0, 3, 1, 2), ref + rowbias.float()[:, :, None, None])
    # weight gradient
    dy = bf(torch.randn(B, cout, OH, OH, device="cuda"))
    xr = x.float().cpu().requires_grad_(True)
    wr = w.float().cpu().requires_grad_(True)
    F.conv2d(xr, wr, stride=stride, padding=pad).backward(dy.float().cpu())
    dw = torch.empty(cout, cin, ks, ks, device="cuda")
    dyn = dy.permute(0, 2, 3, 1).contiguous()
    k.conv_wgrad(dyn, cout, xn, B, H, H, cin, cin, cout, ks, ks, stride, pad, dw, OH, OH)
    close(dw, wr.grad.cuda(), 2e-3)


@pytest.mark.parametrize("B,H,cin,cout", [(2, 4, 16, 24), (3, 8, 64, 32)])
def test_convT_phases(B, H, cin, cout):
    k, L = _k()
    torch.manual_seed(4)
    x = bf(torch.randn(B, cin, H, H, device="cuda"))
    w = bf(torch.randn(cin, cout, 4, 4, device="cuda") * 0.1)
    ref = F.conv_transpose2d(x.float().cpu(), w.float().cpu(), stride=2, padding=1).cuda()
    xn = x.permute(0, 2, 3, 1).contiguous()
    wph = []
    for ph in range(2):
        for pw in range(2):
            th, tw = k.phase_taps(ph), k.phase_taps(pw)
            sub = w[:, :, th][:, :, :, tw]            # (cin, cout, 2, 2) [a][b]
            wph.append(sub.permute(1, 2, 3, 0).contiguous())  # [cout][a][b][cin]
    out = torch.empty(B, 2 * H, 2 * H, cout, device="cuda", dtype=torch.bfloat16)
    k.convT_fwd_phases(xn, B, H, H, cin, cin, wph, cout, out, cout)
    close(out.permute(0, 3, 1, 2), ref)


@pytest.mark.parametrize("splits", [0, 4])
def test_rowmajor_nk_tile192(splits):
    """32700 x 384 picks the 128 x 192 tile (one round of 512 workgroups); ragged M and K, bias + residual
    epilogue, and a forced split-K (raw slabs + reducer) on the same tile."""
    k, L = _k()
    torch.manual_seed(5)
    M, N, K = 32700, 384, 200
    a = bf(torch.randn(M, K, device="cuda"))
    w = bf(torch.randn(N, K, device="cuda"))
    bias = torch.randn(N, device="cuda")
    res = bf(torch.randn(M, N, device="cuda"))
    c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    saved = k.TUNED
    try:
        if splits:
            d = k.GemmDesc()
            d.m, d.n, d.k, d.a_mode, d.b_mode = M, N, K, L.A_ROWMAJOR, L.B_NK
            k.TUNED = {k.gemm_key(d): splits}
        k.gemm(M, N, K, a, L.A_ROWMAJOR, K, w, L.B_NK, K, c, N, bias=bias, resid=res, ldr=N)
    finally:
        k.TUNED = saved
    close(c, a.float() @ w.float().t() + bias + res.float())


def test_conv_fwd_tile192():
    k, L = _k()
    torch.manual_seed(6)
    B, H, cin, cout = 32, 32, 64, 384
    x = bf(torch.randn(B, cin, H, H, device="cuda"))
    w = bf(torch.randn(cout, cin, 3, 3, device="cuda") * 0.1)
    ref = F.conv2d(x.float().cpu(), w.float().cpu(), padding=1).cuda()
    xn = x.permute(0, 2, 3, 1).contiguous()
    wpk = w.permute(0, 2, 3, 1).contiguous()
    out = torch.empty(B, H, H, cout, device="cuda", dtype=torch.bfloat16)
    k.conv_fwd(xn, B, H, H, cin, cin, wpk, cout, 3, 3, 1, 1, out, cout)
    close(out.permute(0, 3, 1, 2), ref)


@pytest.mark.parametrize("M,N,K,group,splits", [(136, 264, 200, 50, 0), (384, 384, 32768, 1024, 0),
                                                 (512, 512, 2048, 64, 1), (128, 128, 4096, 256, 8)])
def test_wgrad_with_fused_bias_and_group_sums(M, N, K, group, splits):
    """Weight-gradient GEMM (col-major A = dY^T) with the bias gradient (row sums of A over k) and per-group sums
    (per-sample time-embedding gradient) produced by the same launch through synthesised B columns; with and
    without split-K (the reducer applies the same routing)."""
    k, L = _k()
    torch.manual_seed(7)
    dy = bf(torch.randn(K, M, device="cuda"))
    x = bf(torch.randn(K, N, device="cuda"))
    out = torch.empty(M, N, device="cuda")
    bg = torch.full((M,), float("nan"), device="cuda")
    bg2 = torch.full((M,), float("nan"), device="cuda")
    G = (K + group - 1) // group
    gs = torch.zeros(G, M + 16, device="cuda", dtype=torch.bfloat16)[:, 8:8 + M]
    if splits:
        k.TUNED = {k.gemm_key(_desc(k, L, M, N, K)): splits}
    try:
        k.gemm(M, N, K, dy, L.A_COLMAJOR, M, x, L.B_KN, N, out, N, sum_out=bg, sum_out2=bg2, gsum=gs, sum_group=group)
    finally:
        k.TUNED = None
    torch.cuda.synchronize()
    close(out, dy.float().t() @ x.float(), 2e-3)
    ref = dy.float().sum(0)
    close(bg, ref, 1e-5)
    assert torch.equal(bg, bg2)
    gref = torch.stack([dy.float()[g * group:(g + 1) * group].sum(0) for g in range(G)])
    close(gs, gref, 1e-2)


def _desc(k, L, M, N, K):
    d = L.GemmDesc()
    d.m, d.n, d.k, d.a_mode, d.b_mode = M, N, K, L.A_COLMAJOR, L.B_KN
    return d


def test_conv_wgrad_with_fused_bias_and_group_sums():
    """conv_wgrad (implicit im2col B) with the conv-bias and per-sample sums of dY fused, at a non-power-of-two
    grid (B=3, 12x20)."""
    k, L = _k()
    torch.manual_seed(8)
    B, H, W, C, O = 3, 12, 20, 32, 48
    x = bf(torch.randn(B * H * W, C, device="cuda"))
    dy = bf(torch.randn(B * H * W, O, device="cuda"))
    dw = torch.empty(O, C, 3, 3, device="cuda")
    bg = torch.empty(O, device="cuda")
    gs = torch.empty(B, O, device="cuda", dtype=torch.bfloat16)
    k.conv_wgrad(dy, O, x, B, H, W, C, C, O, 3, 3, 1, 1, dw, H, W, bias_grad=bg, group_sums=gs)
    torch.cuda.synchronize()
    xn = x.float().view(B, H, W, C).permute(0, 3, 1, 2)
    dyn = dy.float().view(B, H, W, O).permute(0, 3, 1, 2)
    ref = torch.nn.grad.conv2d_weight(xn, (O, C, 3, 3), dyn, padding=1)
    close(dw, ref, 2e-3)
    close(bg, dyn.sum((0, 2, 3)), 1e-5)
    close(gs, dyn.sum((2, 3)), 1e-2)


@pytest.mark.parametrize("G,M,N,K,bias", [(3, 4096, 384, 384, True), (6, 512, 512, 512, True), (2, 2464, 768, 384, False),
                                         (8, 1024, 128, 128, True)])
def test_grouped_weight_gradients_match_single_launches(G, M, N, K, bias):
    """sdmi_gemm_grouped: G same-shape weight gradients in one launch give, per problem, exactly the single launch's
    result at the same split count and mainloop (weights and bias sums bitwise), with and without split-K."""
    from sdmi import _lib, kernels as K_
    import ctypes
    saved, K_.TUNED = K_.TUNED, {}  # built-in heuristics on both sides (no per-shape table hints)
    try:
        _grouped_check(G, M, N, K, bias, _lib, K_, ctypes)
    finally:
        K_.TUNED = saved


def _grouped_check(G, M, N, K, bias, _lib, K_, ctypes):
    g = torch.Generator().manual_seed(11)
    items, ref = [], []
    for i in range(G):
        dy = (torch.randn(M, N, generator=g) * 0.5).to(torch.bfloat16).cuda()
        x = torch.randn(M, K, generator=g).to(torch.bfloat16).cuda()
        out = torch.full((N, K), float("nan"), device="cuda")
        bg = torch.full((N,), float("nan"), device="cuda") if bias else None
        items.append((dy, x, out, bg))
    K_.linear_wgrad_grouped(items)
    # the same split count the grouped launch used, one problem at a time
    d = K_.GemmDesc()
    d.m, d.n, d.k = N, K, M
    d.a_mode, d.b_mode = _lib.A_COLMAJOR, _lib.B_KN
    d.a, d.lda, d.b, d.ldb = items[0][0].data_ptr(), N, items[0][1].data_ptr(), K
    d.c, d.ldc, d.c_f32, d.alpha = items[0][2].data_ptr(), K, 1, 1.0
    d.sum_out = K_._p(items[0][3])
    d.variant_hint = K_.GROUPED_VARIANT  # the grouped launch's mainloop
    descs = (K_.GemmDesc * G)(*([d] * G))
    sp = ctypes.c_int(0)
    wsb = ctypes.c_size_t(0)
    _lib.check(_lib.lib().sdmi_gemm_grouped_plan(descs, G, ctypes.byref(sp), ctypes.byref(wsb)), "plan")
    torch.cuda.synchronize()
    for dy, x, out, bg in items:
        o1 = torch.empty_like(out)
        b1 = torch.empty_like(bg) if bias else None
        K_.gemm(N, K, M, dy, _lib.A_COLMAJOR, N, x, _lib.B_KN, K, o1, K, sum_out=b1)  # heuristic / tuned split
        fp = (dy.float().t() @ x.float())
        assert (out - fp).abs().max().item() <= 2e-3 * fp.abs().max().item() + 1e-3
        if bias:
            assert (bg - dy.float().sum(0)).abs().max().item() <= 1e-2 * (1 + dy.float().sum(0).abs().max().item())
    # bitwise vs single launches forced to the grouped split count
    for dy, x, out, bg in items:
        o1 = torch.empty_like(out)
        b1 = torch.empty_like(bg) if bias else None
        dd = K_.GemmDesc.from_buffer_copy(d)
        dd.a, dd.b, dd.c, dd.sum_out = dy.data_ptr(), x.data_ptr(), o1.data_ptr(), K_._p(b1)
        dd.splits_hint = sp.value
        s1 = ctypes.c_int(0)
        w1 = ctypes.c_size_t(0)
        _lib.check(_lib.lib().sdmi_gemm_plan(ctypes.byref(dd), ctypes.byref(s1), ctypes.byref(w1)), "plan1")
        assert s1.value == sp.value
        ws = torch.empty(max(1, w1.value // 4), device="cuda")
        _lib.check(_lib.lib().sdmi_gemm(ctypes.byref(dd), ws.data_ptr(), w1.value, K_._stream()), "gemm1")
        torch.cuda.synchronize()
        assert torch.equal(o1, out)
        if bias:
            assert torch.equal(b1, bg)
