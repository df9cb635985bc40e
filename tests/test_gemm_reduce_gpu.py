"""Weight-gradient GEMMs with fused reduction outputs (bias sums, second bias, per-sample group sums -- the bias and
time-embedding gradients of /root/reference/models/blocks.py:45-74,116-120) on every mainloop and split count:
run-to-run bitwise determinism (3 repeats) and accuracy against a torch fp32 reference of the same op.

Round 4 found the LDS-DMA mainloop's split-K slabs of these launches racy (profiles/r04_gsum_probe.txt): the last
column tile's padding stored zero accumulators into the reduction columns of the slab. These cases pin the fix; the
shapes include the probe's failing ones (N = 9 * C not a multiple of the column tile)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

# tuned-table mainloop ids (sdmi/tuned_gemm.json): 1 register staging, 2 / 3 / 5 / 6 LDS-DMA rings (3 falls back to 2
# where reduction columns ride along), 4 = 128 x {256, 384} tiles on 8 waves, 11 = two k-groups of 4 waves per tile
VARIANTS = (1, 2, 3, 5, 6, 11)
SPLITS = (1, 2, 4, 8)


def _forced(monkeypatch, K, splits, variant):
    monkeypatch.setattr(K, "TUNED", {"__all__": [splits, variant]})
    monkeypatch.setattr(K, "gemm_key", lambda d: "__all__")


def _relerr(a, ref):
    return ((a.float() - ref).abs().max() / (ref.abs().max() + 1e-9)).item()


# (B, H, C, O): conv3x3 weight gradients, dW [O][9 C]; (2, 32, 32, 64) / (2, 16, 64, 64) / (4, 8, 32, 32) are the
# round-4 probe's failing shapes
CONV_SHAPES = [(2, 32, 32, 64), (2, 16, 64, 64), (4, 8, 32, 32), (2, 4, 128, 128), (3, 8, 16, 48)]


@pytest.mark.parametrize("gsum", [False, True], ids=["bias", "bias+gsum"])
@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("shape", CONV_SHAPES, ids=lambda s: "B{}H{}C{}O{}".format(*s))
def test_conv_wgrad_reductions_deterministic(monkeypatch, shape, variant, gsum):
    from sdmi import kernels as K
    B, H, C, O = shape
    g = torch.Generator().manual_seed(5 + B * H + C)
    x = torch.randn(B * H * H, C, generator=g).to(torch.bfloat16).cuda()
    dy = (torch.randn(B * H * H, O, generator=g) * 0.5).to(torch.bfloat16).cuda()
    xn = x.float().view(B, H, H, C).permute(0, 3, 1, 2)
    dyn = dy.float().view(B, H, H, O).permute(0, 3, 1, 2)
    wref = torch.nn.grad.conv2d_weight(xn, (O, C, 3, 3), dyn, padding=1)
    gref = dyn.sum((2, 3))
    bref = gref.sum(0)
    for sp in SPLITS:
        _forced(monkeypatch, K, sp, variant)
        outs = []
        for _ in range(3):
            dw = torch.full((O, C, 3, 3), float("nan"), device="cuda")
            bg = torch.full((O,), float("nan"), device="cuda")
            bg2 = torch.full((O,), float("nan"), device="cuda")
            gs = torch.full((B, O), float("nan"), device="cuda", dtype=torch.bfloat16) if gsum else None
            K.conv_wgrad(dy, O, x, B, H, H, C, C, O, 3, 3, 1, 1, dw, H, H, bias_grad=bg, bias_grad2=bg2, group_sums=gs)
            outs.append((dw, bg, bg2) + ((gs,) if gsum else ()))
        torch.cuda.synchronize()
        o0 = outs[0]
        tag = f"splits={sp} variant={variant}"
        for o in outs[1:]:
            for a, b in zip(o, o0):
                assert torch.equal(a, b), f"not run-to-run deterministic ({tag})"
        assert _relerr(o0[0], wref) < 2e-3, tag
        assert _relerr(o0[1], bref) < 1e-5, tag
        assert torch.equal(o0[1], o0[2]), tag
        if gsum:
            assert _relerr(o0[3], gref) < 1e-2, tag


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("M,N,K,group", [(2048, 288, 384, 1024), (512, 136, 264, 64), (4096, 320, 64, 256)])
def test_linear_wgrad_reductions_deterministic(monkeypatch, M, N, K, group, variant):
    """Linear weight gradients (col-major A = dY, row-major B = X) with bias + group sums; N is the output-channel
    count (rows of dW), K the input features (columns of dW, not a multiple of 128)."""
    from sdmi import kernels as Kn
    g = torch.Generator().manual_seed(M + N + K)
    dy = (torch.randn(M, N, generator=g) * 0.5).to(torch.bfloat16).cuda()
    x = torch.randn(M, K, generator=g).to(torch.bfloat16).cuda()
    G = M // group
    wref = dy.float().t() @ x.float()
    gref = dy.float().view(G, group, N).sum(1)
    for sp in SPLITS:
        _forced(monkeypatch, Kn, sp, variant)
        outs = []
        for _ in range(3):
            out = torch.full((N, K), float("nan"), device="cuda")
            bg = torch.full((N,), float("nan"), device="cuda")
            gs = torch.full((G, N), float("nan"), device="cuda", dtype=torch.bfloat16)
            Kn.linear_wgrad(dy, x, out, bias_grad=bg, group_sums=gs, group=group)
            outs.append((out, bg, gs))
        torch.cuda.synchronize()
        tag = f"splits={sp} variant={variant}"
        for o in outs[1:]:
            for a, b in zip(o, outs[0]):
                assert torch.equal(a, b), f"not run-to-run deterministic ({tag})"
        assert _relerr(outs[0][0], wref) < 2e-3, tag
        assert _relerr(outs[0][1], gref.sum(0)) < 1e-5, tag
        assert _relerr(outs[0][2], gref) < 1e-2, tag


@pytest.mark.parametrize("variant", (2, 3, 5, 11))
@pytest.mark.parametrize("G,M,N,K,splits", [(2, 8192, 288, 288, 24), (3, 8192, 288, 1152, 12), (6, 512, 512, 512, 8),
                                             (7, 2048, 136, 264, 4)])
def test_grouped_wgrad_bias_deterministic(monkeypatch, G, M, N, K, splits, variant):
    """Grouped weight gradients with bias sums on the LDS-DMA mainloop at the split counts the tuned table hands
    them (DiT 2- / 3-layer groups: the single problem's 24 / 12 splits shared out), repeated: bitwise deterministic,
    and each problem matches a torch fp32 reference."""
    from sdmi import kernels as Kn
    monkeypatch.setattr(Kn, "TUNED", {"__all__": splits})
    monkeypatch.setattr(Kn, "gemm_key", lambda d: "__all__")
    monkeypatch.setattr(Kn, "GROUPED_VARIANT", variant)
    g = torch.Generator().manual_seed(G * 31 + N)
    data = [((torch.randn(M, N, generator=g) * 0.5).to(torch.bfloat16).cuda(),
             torch.randn(M, K, generator=g).to(torch.bfloat16).cuda()) for _ in range(G)]
    runs = []
    for _ in range(3):
        items = [(dy, x, torch.full((N, K), float("nan"), device="cuda"), torch.full((N,), float("nan"), device="cuda"))
                 for dy, x in data]
        Kn.linear_wgrad_grouped(items)
        runs.append(items)
    torch.cuda.synchronize()
    for r in runs[1:]:
        for (_, _, o, b), (_, _, o0, b0) in zip(r, runs[0]):
            assert torch.equal(o, o0) and torch.equal(b, b0), "grouped launch not run-to-run deterministic"
    for dy, x, o, b in runs[0]:
        assert _relerr(o, dy.float().t() @ x.float()) < 2e-3
        assert _relerr(b, dy.float().sum(0)) < 1e-5


@pytest.mark.parametrize("splits", (1, 2, 3, 5))
@pytest.mark.parametrize("M,N,K", [(136, 264, 200), (384, 512, 192), (128, 1152, 4160), (256, 384, 64)])
def test_kgroup_mainloop_plain_colmajor(monkeypatch, M, N, K, splits):
    """Variant 11 (two k-groups per workgroup, interleaved k-tiles, accumulators summed through LDS in group order) on
    plain col-major weight-gradient GEMMs, including splits whose k-tile count is odd or smaller than the group count
    (one group idles through its barriers): bitwise deterministic over repeats and within fp32 tolerance."""
    from sdmi import kernels as Kn, _lib as L
    _forced(monkeypatch, Kn, splits, 11)
    g = torch.Generator().manual_seed(M * 7 + N + K)
    at = torch.randn(K, M, generator=g).to(torch.bfloat16).cuda()
    b = torch.randn(K, N, generator=g).to(torch.bfloat16).cuda()
    outs = []
    for _ in range(3):
        c = torch.full((M, N), float("nan"), device="cuda")
        Kn.gemm(M, N, K, at, L.A_COLMAJOR, M, b, L.B_KN, N, c, N)
        outs.append(c)
    torch.cuda.synchronize()
    assert all(torch.equal(o, outs[0]) for o in outs[1:])
    assert _relerr(outs[0], at.float().t() @ b.float()) < 2e-3


@pytest.mark.parametrize("splits", (1, 2, 3))
def test_kgroup_mainloop_rowmajor_and_conv(monkeypatch, splits):
    """Variant 11 on the forward / data-gradient operand modes: a ragged row-major linear with bias + residual, an
    implicit-GEMM 3x3 conv with cin % 64 == 0 (incremental tap state advanced per k-group), one with cin = 32 (general
    gather), and a conv with the K-concatenated 1x1 second source; repeated bitwise and against torch fp32."""
    import torch.nn.functional as F
    from sdmi import kernels as Kn, _lib as L
    _forced(monkeypatch, Kn, splits, 11)
    g = torch.Generator().manual_seed(41 + splits)
    bf = torch.bfloat16
    M, N, Kd = 300, 200, 136
    a = torch.randn(M, Kd, generator=g).to(bf).cuda()
    w = torch.randn(N, Kd, generator=g).to(bf).cuda()
    bias = torch.randn(N, generator=g).cuda()
    res = torch.randn(M, N, generator=g).to(bf).cuda()
    outs = []
    for _ in range(3):
        c = torch.full((M, N), float("nan"), device="cuda")
        Kn.gemm(M, N, Kd, a, L.A_ROWMAJOR, Kd, w, L.B_NK, Kd, c, N, bias=bias, resid=res, ldr=N)
        outs.append(c)
    torch.cuda.synchronize()
    assert all(torch.equal(o, outs[0]) for o in outs[1:])
    assert _relerr(outs[0], a.float() @ w.float().t() + bias + res.float()) < 2e-3
    for (B, H, cin, cout) in ((2, 8, 64, 128), (3, 8, 32, 64)):
        x = torch.randn(B, cin, H, H, generator=g).to(bf)
        wt = (torch.randn(cout, cin, 3, 3, generator=g) * 0.1).to(bf)
        ref = F.conv2d(x.float(), wt.float(), padding=1).cuda()
        xn = x.permute(0, 2, 3, 1).contiguous().cuda()
        wpk = wt.permute(0, 2, 3, 1).contiguous().cuda()
        outs = []
        for _ in range(3):
            y = torch.full((B, H, H, cout), float("nan"), device="cuda")
            Kn.conv_fwd(xn, B, H, H, cin, cin, wpk, cout, 3, 3, 1, 1, y, cout)
            outs.append(y)
        torch.cuda.synchronize()
        assert all(torch.equal(o, outs[0]) for o in outs[1:])
        assert _relerr(outs[0].permute(0, 3, 1, 2), ref) < 2e-3
    # conv + fused 1x1 of a second source (the resnet's conv2 + residual conv): W = [W3x3 | W1x1] along K
    B, H, cin, cin2, cout = 2, 8, 64, 128, 64
    x = torch.randn(B, cin, H, H, generator=g).to(bf)
    x2 = torch.randn(B, cin2, H, H, generator=g).to(bf)
    w3 = (torch.randn(cout, cin, 3, 3, generator=g) * 0.1).to(bf)
    w1 = (torch.randn(cout, cin2, 1, 1, generator=g) * 0.1).to(bf)
    ref = (F.conv2d(x.float(), w3.float(), padding=1) + F.conv2d(x2.float(), w1.float())).cuda()
    wcat = torch.cat([w3.permute(0, 2, 3, 1).reshape(cout, -1), w1.reshape(cout, -1)], 1).contiguous().cuda()
    xn, x2n = x.permute(0, 2, 3, 1).contiguous().cuda(), x2.permute(0, 2, 3, 1).contiguous().cuda()
    y = torch.full((B, H, H, cout), float("nan"), device="cuda")
    Kn.conv_fwd(xn, B, H, H, cin, cin, wcat, cout, 3, 3, 1, 1, y, cout, x2=x2n.view(-1, cin2), cin2=cin2)
    torch.cuda.synchronize()
    assert _relerr(y.permute(0, 3, 1, 2), ref) < 2e-3
