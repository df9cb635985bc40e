"""Leaf-path glue kernels (csrc/leafops.hip) against the aten ops the reference writes between its layers:
F.interpolate nearest (unet_cond_base.py:132, transformer.py:169), torch.cat along channels and its gradient split
(unet_cond_base.py:136, blocks.py:463-464), the DiT adaLN modulation / gated residual and their gradients
(transformer_layer.py:86-100, transformer.py:205-207), and the need_weights attention map
(multihead_attention.py:107-118)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _lf():
    from sdmi import leaf as LF
    return LF


@pytest.mark.parametrize("shape,size", [((2, 18, 64, 64), (32, 32)), ((3, 5, 48, 40), (32, 32)),
                                        ((2, 3, 7, 9), (32, 20)), ((1, 18, 512, 512), (32, 32))])
def test_resize_nearest_bit_exact(shape, size):
    g = torch.Generator().manual_seed(1)
    x = torch.randn(*shape, generator=g).cuda()
    ref = torch.nn.functional.interpolate(x, size=size)
    assert torch.equal(_lf().resize_nearest(x, size), ref)


def test_cat_channels_and_gradient_split():
    g = torch.Generator().manual_seed(2)
    a = torch.randn(3, 4, 8, 8, generator=g).cuda().requires_grad_(True)
    b = torch.randn(3, 7, 8, 8, generator=g).cuda().requires_grad_(True)
    out = _lf().cat_channels([a, b])
    assert torch.equal(out, torch.cat([a, b], dim=1))
    w = torch.randn(out.shape, generator=g).cuda()
    (out * w).sum().backward()
    assert torch.equal(a.grad, w[:, :4]) and torch.equal(b.grad, w[:, 4:])


@pytest.mark.parametrize("mode", ["modulation", "gated_residual"])
def test_modulate_forward_backward(mode):
    LF = _lf()
    g = torch.Generator().manual_seed(3)
    B, N, C = 3, 37, 72
    x = torch.randn(B, N, C, generator=g).cuda().requires_grad_(True)
    table = torch.randn(B, 6 * C, generator=g).cuda().requires_grad_(True)  # an adaLN output, chunked as the model does
    r = torch.randn(B, N, C, generator=g).cuda().requires_grad_(True)
    w = torch.randn(B, N, C, generator=g).cuda()

    def run(ours):
        s, t = table.chunk(6, dim=1)[1], table.chunk(6, dim=1)[0]
        if mode == "modulation":
            y = LF.modulate(x, s, t) if ours else x * (1 + s.unsqueeze(1)) + t.unsqueeze(1)
        else:
            y = LF.modulate(x, s, r=r, alpha=0.0) if ours else r + s.unsqueeze(1) * x
        (y * w).sum().backward()
        grads = [v.grad.clone() for v in (x, table, r) if v.grad is not None]
        for v in (x, table, r):
            v.grad = None
        return y.detach(), grads

    y1, g1 = run(True)
    y0, g0 = run(False)
    assert (y1 - y0).abs().max().item() <= 1e-5
    assert len(g1) == len(g0)
    for a, b in zip(g1, g0):
        assert (a - b).abs().max().item() <= 1e-4 * max(1.0, b.abs().max().item())


@pytest.mark.parametrize("average", [True, False])
@pytest.mark.parametrize("N,S,H,d", [(64, 77, 3, 32), (256, 256, 9, 32), (16, 1024, 2, 8)])
def test_attention_map(average, N, S, H, d):
    LF = _lf()
    g = torch.Generator().manual_seed(4)
    B = 2
    q = torch.randn(B, N, H * d, generator=g).cuda()
    k = torch.randn(B, S, H * d, generator=g).cuda()
    scaling = d ** -0.5
    qh = q.reshape(B, N, H, d).transpose(1, 2)
    kh = k.reshape(B, S, H, d).transpose(1, 2)
    ref = torch.softmax(qh @ kh.transpose(-2, -1) * scaling, dim=-1)
    ref = ref.mean(dim=1) if average else ref
    out = LF.attention_map(q, k, H, scaling, average)
    assert out.shape == ref.shape
    assert (out - ref).abs().max().item() <= 2e-6


def test_custom_mha_need_weights_matches_reference_math():
    """CustomMultiheadAttention(need_weights=True) returns the reference's head-averaged map next to its output."""
    from models.multihead_attention import CustomMultiheadAttention
    torch.manual_seed(5)
    m = CustomMultiheadAttention(96, 3, batch_first=True).cuda()
    x = torch.randn(2, 50, 96, device="cuda")
    ctx = torch.randn(2, 77, 96, device="cuda")
    out, wts = m(x, ctx, ctx, need_weights=True)
    from sdmi import leaf as LF
    q, k = LF.call(m.q_proj, x), LF.call(m.k_proj, ctx)  # the projections exactly as the module ran them
    qh = q.reshape(2, 50, 3, 32).transpose(1, 2)
    kh = k.reshape(2, 77, 3, 32).transpose(1, 2)
    ref = torch.softmax(qh @ kh.transpose(-2, -1) * m.scaling, dim=-1).mean(dim=1)
    assert wts.shape == (2, 50, 77) and (wts - ref).abs().max().item() <= 1e-5
    assert torch.isfinite(out).all()
