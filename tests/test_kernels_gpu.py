"""GPU numerics of the GroupNorm, attention and small fused kernels against torch fp32 references
of the same ops on bf16-rounded inputs.  Tolerances: bf16 output rounding (~4e-3 relative) plus
fp32 reduction-order differences."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def K():
    from sdmi import kernels
    return kernels


def bf(t):
    return t.to(torch.bfloat16)


def relerr(a, b):
    return ((a.float() - b.float()).abs().max() / (b.float().abs().max() + 1e-12)).item()


@pytest.mark.parametrize("B,H,C,G,silu", [(2, 8, 64, 32, True), (3, 16, 384, 32, True), (2, 4, 768, 32, False),
                                          (1, 32, 96, 32, True),
                                          # single-pass shapes of the B=32 step: 1024-thread 24-channel strips (C=384 at
                                          # 32^2), 8-channel strips (C=256), 64-thread workgroups (4^2), ragged P
                                          (32, 32, 384, 32, True), (32, 32, 256, 32, False), (32, 4, 768, 32, True),
                                          (4, 30, 384, 32, True), (32, 16, 512, 32, True),
                                          (1024, 2, 512, 32, True)])  # 256-channel strips on 64 threads
def test_groupnorm_fwd_bwd(B, H, C, G, silu):
    k = K()
    torch.manual_seed(0)
    P = H * H
    x = bf(torch.randn(B, P, C, device="cuda") * 2 + 0.5)
    gamma = torch.randn(C, device="cuda") * 0.1 + 1
    beta = torch.randn(C, device="cuda") * 0.1
    dy = bf(torch.randn(B, P, C, device="cuda"))
    # reference on the CPU in float64: aten's ROCm group_norm backward returns wrong weight / bias gradients for
    # batches >= 256 on this image (measured: half the per-channel sums; the CPU kernels agree with ours)
    xr = x.double().cpu().permute(0, 2, 1).clone().requires_grad_(True)  # (B, C, P)
    gr = gamma.double().cpu().requires_grad_(True)
    br = beta.double().cpu().requires_grad_(True)
    yr = F.group_norm(xr, G, gr, br, eps=1e-5)
    if silu:
        yr = F.silu(yr)
    yr.backward(dy.double().cpu().permute(0, 2, 1))
    xg, gg, bg_, yref = xr.grad.float().cuda(), gr.grad.float().cuda(), br.grad.float().cuda(), yr.detach().float().cuda()
    x2 = x.view(B * P, C)
    tab = k.gn_stats(x2, B, P, C, G, gamma, beta)
    y = torch.empty_like(x2)
    k.gn_apply(x2, tab, B, P, C, silu, y)
    assert relerr(y.view(B, P, C).permute(0, 2, 1), yref) < 1e-2
    dx = torch.empty_like(x2)
    dg = torch.empty(C, device="cuda")
    db = torch.empty(C, device="cuda")
    k.gn_bwd(x2, dy.view(B * P, C), dx, tab, gamma, B, P, C, G, silu, dg, db)
    assert relerr(dx.view(B, P, C).permute(0, 2, 1), xg) < 2e-2
    assert relerr(dg, gg) < 1e-2
    assert relerr(db, bg_) < 1e-2
    # gn_fwd (single pass for P <= 256, stats + apply beyond): same output and table
    y2 = torch.empty_like(x2)
    tab2 = k.gn_fwd(x2, B, P, C, G, gamma, beta, silu, y2)
    assert relerr(y2.view(B, P, C).permute(0, 2, 1), yref) < 1e-2
    assert relerr(tab2, tab) < 1e-4
    # in-place backward (dx aliases dy) with an addend, as the resnet blocks call it
    add = bf(torch.randn(B * P, C, device="cuda"))
    buf = dy.view(B * P, C).clone()
    k.gn_bwd(x2, buf, buf, tab2, gamma, B, P, C, G, silu, None, None, addend=add)
    assert relerr(buf.view(B, P, C).permute(0, 2, 1), xg + add.float().view(B, P, C).permute(0, 2, 1)) < 2e-2


class _AllSplit(dict):
    """tuned-table stand-in: every GEMM launch asks for `n` split-K slices"""

    def __init__(self, n):
        super().__init__()
        self.n = n

    def __bool__(self):
        return True

    def get(self, key, default=0):
        return self.n


# B, P (pixels per sample), C, producer ("conv": 3x3 implicit-GEMM data gradient, "linear": in-projection data gradient),
# silu; the cond-UNet's GroupNorm inputs: 32^2 / 16^2 / 8^2 / 4^2 levels
@pytest.mark.parametrize("B,H,C,prod,silu", [(4, 32, 384, "conv", True), (4, 16, 512, "linear", False),
                                             (8, 8, 768, "conv", True), (32, 4, 512, "conv", True),
                                             (32, 4, 512, "linear", False), (3, 16, 96, "conv", True)])
@pytest.mark.parametrize("splits", [1, 4])
def test_groupnorm_bwd_from_gemm_statistics(B, H, C, prod, silu, splits, monkeypatch):
    """GroupNorm backward whose Σdz / Σdz·x̂ come out of the producing data-gradient GEMM (sdmi_gemm_desc::gn_part:
    the unsplit epilogue and the split-K reducer) followed by the streaming sdmi_gn_bwd_part, against the
    self-contained sdmi_gn_bwd on the same dy: the GEMM output is bitwise unchanged, dx / dgamma / dbeta agree to fp32
    summation order (the partials are summed per segment, then over segments)."""
    k = K()
    monkeypatch.setattr(k, "TUNED", _AllSplit(splits))
    torch.manual_seed(1)
    P, G = H * H, 32
    M = B * P
    x = bf(torch.randn(M, C, device="cuda") * 2 + 0.5)
    gamma = torch.randn(C, device="cuda") * 0.1 + 1
    beta = torch.randn(C, device="cuda") * 0.1
    y = torch.empty_like(x)
    tab = k.gn_fwd(x, B, P, C, G, gamma, beta, silu, y)
    if prod == "conv":  # dy = conv3x3 data gradient of an upstream gradient (cout = 256) through packed weights
        cu = 256
        g_up = bf(torch.randn(M, cu, device="cuda"))
        wd = bf(torch.randn(C, 9 * cu, device="cuda") * 0.02)
        run = lambda out, gn: k.conv_fwd(g_up, B, H, H, cu, cu, wd, C, 3, 3, 1, 1, out, C, gn=gn)  # noqa: E731
    else:
        n3 = 3 * C
        g_up = bf(torch.randn(M, n3, device="cuda"))
        w = bf(torch.randn(n3, C, device="cuda") * 0.05)
        run = lambda out, gn: k.linear_dgrad(g_up, w, out, gn=gn)  # noqa: E731
    dy_ref = torch.empty(M, C, dtype=torch.bfloat16, device="cuda")
    run(dy_ref, None)
    dy = torch.empty_like(dy_ref)
    req = k.gn_request(x, tab, P, C, silu)
    assert req is not None
    run(dy, req)
    torch.cuda.synchronize()
    assert torch.equal(dy, dy_ref)
    assert req["rb"] == (16 if splits > 1 else min(64, P))
    add = bf(torch.randn(M, C, device="cuda"))
    dx_ref, dx = torch.empty_like(x), torch.empty_like(x)
    dg_ref, db_ref, dg, db = (torch.empty(C, device="cuda") for _ in range(4))
    k.gn_bwd(x, dy_ref, dx_ref, tab, gamma, B, P, C, G, silu, dg_ref, db_ref, addend=add)
    k.gn_bwd(x, dy, dx, tab, gamma, B, P, C, G, silu, dg, db, addend=add, gn=req)
    torch.cuda.synchronize()
    assert relerr(dx, dx_ref) < 2e-3, relerr(dx, dx_ref)
    assert relerr(dg, dg_ref) < 1e-4 and relerr(db, db_ref) < 1e-4, (relerr(dg, dg_ref), relerr(db, db_ref))
    # deterministic: the same launches again give the same bits
    dx2 = torch.empty_like(x)
    req2 = k.gn_request(x, tab, P, C, silu)
    run(dy, req2)
    k.gn_bwd(x, dy, dx2, tab, gamma, B, P, C, G, silu, dg, db, addend=add, gn=req2)
    torch.cuda.synchronize()
    assert torch.equal(dx2, dx)
    # dgamma / dbeta deferred (per-sample rows, summed by the grouped rows-sum launch): the same bits
    pend = []
    dx3, dg3, db3 = torch.empty_like(x), torch.empty(C, device="cuda"), torch.empty(C, device="cuda")
    req3 = k.gn_request(x, tab, P, C, silu)
    run(dy, req3)
    k.gn_bwd(x, dy, dx3, tab, gamma, B, P, C, G, silu, dg3, db3, addend=add, gn=req3, defer=pend)
    assert len(pend) == 1
    k.gn_rows_sum_grouped(pend)
    torch.cuda.synchronize()
    assert torch.equal(dx3, dx)
    assert relerr(dg3, dg) < 1e-5 and relerr(db3, db) < 1e-5  # the inline tail may group the batch rows differently


@pytest.mark.parametrize("shapes", [[(2, 8, 64)], [(32, 32, 384), (32, 16, 512), (32, 4, 768)],
                                    [(4, 8, 96)] * 17])  # 17 jobs: two grouped launches
def test_groupnorm_bwd_deferred_sums_match_inline(shapes):
    """sdmi_gn_bwd_rows (dgamma / dbeta as per-sample rows, no batch tail) + sdmi_gn_rows_sum_grouped over several
    GroupNorms against the inline sdmi_gn_bwd: dx bitwise equal, dgamma / dbeta to fp32 summation order (the inline
    batch tail of a narrow strip sums interleaved groups of batch rows, the rows sum runs in batch order); the grouped
    launch bitwise equals one sdmi_gn_rows_sum per GroupNorm."""
    k = K()
    torch.manual_seed(2)
    pend, refs, outs = [], [], []
    for B, H, C in shapes:
        P, G = H * H, 32
        x = bf(torch.randn(B * P, C, device="cuda") * 2 + 0.5)
        gamma = torch.randn(C, device="cuda") * 0.1 + 1
        beta = torch.randn(C, device="cuda") * 0.1
        tab = k.gn_fwd(x, B, P, C, G, gamma, beta, True, torch.empty_like(x))
        dy = bf(torch.randn(B * P, C, device="cuda"))
        dx_ref, dx = torch.empty_like(x), torch.empty_like(x)
        dg_ref, db_ref, dg, db = (torch.empty(C, device="cuda") for _ in range(4))
        k.gn_bwd(x, dy, dx_ref, tab, gamma, B, P, C, G, True, dg_ref, db_ref)
        k.gn_bwd(x, dy, dx, tab, gamma, B, P, C, G, True, dg, db, defer=pend)
        refs.append((dx_ref, dg_ref, db_ref))
        outs.append((dx, dg, db))
    assert len(pend) == len(shapes)
    k.gn_rows_sum_grouped(pend)
    single = [(torch.empty_like(dg), torch.empty_like(db)) for (_, dg, db) in outs]
    for (rows, B, C, _, _), (dg1, db1) in zip(pend, single):
        k.gn_rows_sum(rows, B, C, dg1, db1)
    torch.cuda.synchronize()
    for (a, b, c), (a2, b2, c2), (b3, c3) in zip(refs, outs, single):
        assert torch.equal(a2, a)
        assert relerr(b2, b) < 1e-5 and relerr(c2, c) < 1e-5
        assert torch.equal(b3, b2) and torch.equal(c3, c2)


# d = 8, 24, 40 take the forward's ones-column row sum (d % 16 == 8), incl. ragged N and S = 77
@pytest.mark.parametrize("B,Hh,N,S,d", [(2, 16, 64, 64, 8), (2, 16, 256, 256, 24), (1, 16, 16, 77, 32),
                                        (2, 4, 1024, 1024, 16), (2, 16, 64, 77, 48), (1, 8, 100, 100, 64),
                                        (1, 16, 40, 77, 24), (1, 4, 33, 70, 40), (1, 4, 300, 300, 24),
                                        (2, 2, 130, 257, 32)])
@pytest.mark.parametrize("fused", [True, False])
def test_attention_fwd_bwd(B, Hh, N, S, d, fused):
    k = K()
    torch.manual_seed(1)
    C = Hh * d
    q = bf(torch.randn(B * N, C, device="cuda"))
    kk = bf(torch.randn(B * S, C, device="cuda"))
    v = bf(torch.randn(B * S, C, device="cuda"))
    do = bf(torch.randn(B * N, C, device="cuda"))

    def heads(t, L):
        return t.float().view(B, L, Hh, d).transpose(1, 2)

    qr, kr, vr = (heads(q, N).requires_grad_(True), heads(kk, S).requires_grad_(True),
                  heads(v, S).requires_grad_(True))
    att = torch.softmax(qr @ kr.transpose(-1, -2) / math.sqrt(d), -1)
    orf = att @ vr
    orf.backward(heads(do, N))
    o = torch.empty(B * N, C, device="cuda", dtype=torch.bfloat16)
    lse = k.attn_fwd(q, kk, v, o, B, Hh, N, S, d)
    assert relerr(heads(o, N), orf.detach()) < 2e-2
    # base-2 log-sum-exp of the scaled scores, [B*H][N]
    lse_ref = (qr.detach() @ kr.detach().transpose(-1, -2) / math.sqrt(d)).logsumexp(-1) * math.log2(math.e)
    assert (lse.view(-1)[:B * Hh * N] - lse_ref.reshape(-1)).abs().max().item() < 2e-2
    dq = torch.empty_like(q)
    dk = torch.empty_like(kk)
    dv = torch.empty_like(v)
    k.attn_bwd(q, kk, v, o, do, lse, dq, dk, dv, B, Hh, N, S, d, fused=fused)
    assert relerr(heads(dq, N), qr.grad) < 3e-2
    assert relerr(heads(dk, S), kr.grad) < 3e-2
    assert relerr(heads(dv, S), vr.grad) < 3e-2
    if fused:  # the cross-key-block dQ sum is in a fixed order: a second run is bitwise identical
        dq2, dk2, dv2 = torch.empty_like(q), torch.empty_like(kk), torch.empty_like(v)
        k.attn_bwd(q, kk, v, o, do, lse, dq2, dk2, dv2, B, Hh, N, S, d, fused=True)
        assert torch.equal(dq, dq2) and torch.equal(dk, dk2) and torch.equal(dv, dv2)


def test_chan_sum_and_mse():
    k = K()
    torch.manual_seed(2)
    B, P, C = 4, 256, 1536
    dy = bf(torch.randn(B * P, C, device="cuda"))
    per_bc = torch.empty(B, C, device="cuda", dtype=torch.bfloat16)
    per_c = torch.empty(C, device="cuda")
    k.chan_sum(dy, B, P, C, per_bc=per_bc, per_c=per_c)
    ref = dy.float().view(B, P, C).sum(1)
    assert relerr(per_bc, ref) < 1e-2
    assert relerr(per_c, ref.sum(0)) < 1e-4
    pred = torch.randn(B * 1024, 8, device="cuda")
    tgt = torch.randn(B, 4, 32, 32, device="cuda")
    grad = torch.empty(B * 1024, 8, device="cuda", dtype=torch.bfloat16)
    loss = torch.empty(1, device="cuda")
    k.mse(pred, 8, tgt, B, 4, 1024, 1.0, grad, loss)
    p4 = pred.view(B, 32, 32, 8)[..., :4].permute(0, 3, 1, 2)
    assert abs(loss.item() - F.mse_loss(p4, tgt).item()) < 1e-5
    g4 = grad.float().view(B, 32, 32, 8)
    assert relerr(g4[..., :4].permute(0, 3, 1, 2), 2 * (p4 - tgt) / p4.numel()) < 1e-2
    assert g4[..., 4:].abs().max().item() == 0
