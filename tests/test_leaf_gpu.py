"""Leaf-module path (sdmi.leaf; SURVEY.md §8(b) layer-swap rule, cim_qn_train/progressive_qn_train.py:614,638-640):
* every HIP leaf op (Conv2d 3x3 / 1x1 / 4x4-s2 with channel counts not multiples of 8, ConvTranspose2d, Linear
  on 2-D / 3-D inputs, GroupNorm(+SiLU), SiLU, nn.MultiheadAttention self / cross) forward and backward against
  the same torch fp32 op (bf16 operands: max error <= 2e-2 of the output scale, gradient cosine >= 0.999);
* a block called on its own (DownBlock with self + cross attention) against the oracle;
* whole models with every nn.Conv2d / nn.Linear swapped for a subclass exactly the way the CIM tool does it
  (`new.weight = module.weight`): the swapped layers' own forwards run, the rest runs on the HIP leaves, and the
  output / gradients match the oracle (cond UNet) and the reference fixture (VQVAE encode / decode)."""
import copy
import os

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F
from safetensors.torch import load_file

from oracle import sd_oracle as O
from oracle import vqvae_oracle as VO
from tests.golden.configs import SMALL_COND, SMALL_VQVAE

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def cos(a, b):
    a, b = a.reshape(-1).double().cpu(), b.reshape(-1).double().cpu()
    return (a @ b / (a.norm() * b.norm() + 1e-30)).item()


def rel(a, b):
    return ((a.cpu() - b.cpu()).abs().max() / (b.abs().max() + 1e-12)).item()


def _check(mod, inputs, leaf_fn, ref_fn, tol=2e-2):
    """leaf_fn(*gpu inputs) through the HIP leaf path against ref_fn(cpu module copy, *cpu inputs): the torch
    reference runs in fp32 on the host (no MIOpen / hipBLASLt kernel in the comparison)."""
    from sdmi import leaf as LF  # noqa: F401
    xs = [x.clone().cuda().requires_grad_(True) for x in inputs]
    xr = [x.clone().requires_grad_(True) for x in inputs]
    mc = copy.deepcopy(mod).cpu()
    y = leaf_fn(*xs)
    yr = ref_fn(mc, *xr)
    assert rel(y.detach(), yr.detach()) <= tol
    g = torch.randn(yr.shape, generator=torch.Generator().manual_seed(1))
    params = [p for p in mod.parameters()]
    gl = torch.autograd.grad(y, xs + params, g.cuda(), allow_unused=True)
    gr = torch.autograd.grad(yr, xr + [p for p in mc.parameters()], g, allow_unused=True)
    for a, b in zip(gl, gr):
        if b is None:
            continue
        assert a is not None
        assert cos(a, b) >= 0.999, (type(mod).__name__, cos(a, b))


@pytest.mark.parametrize("cin,cout,k,s,p", [(5, 12, 3, 1, 1), (16, 24, 1, 1, 0), (16, 16, 4, 2, 1), (18, 32, 1, 1, 0)])
def test_conv2d_leaf(cin, cout, k, s, p):
    from sdmi import leaf as LF
    torch.manual_seed(0)
    m = nn.Conv2d(cin, cout, k, s, p).cuda()
    x = torch.randn(2, cin, 12, 10)
    _check(m, [x], lambda a: LF.conv2d(m, a), lambda m_, a: F.conv2d(a, m_.weight, m_.bias, s, p))


def test_conv_transpose_linear_gn_silu_leaves():
    from sdmi import leaf as LF
    torch.manual_seed(1)
    ct = nn.ConvTranspose2d(16, 16, 4, 2, 1).cuda()
    _check(ct, [torch.randn(2, 16, 6, 5)], lambda a: LF.conv_transpose2d(ct, a),
           lambda m_, a: F.conv_transpose2d(a, m_.weight, m_.bias, 2, 1))
    lin = nn.Linear(24, 40).cuda()
    _check(lin, [torch.randn(6, 24)], lambda a: LF.linear(lin, a), lambda m_, a: F.linear(a, m_.weight, m_.bias))
    _check(lin, [torch.randn(2, 7, 24)], lambda a: LF.linear(lin, a), lambda m_, a: F.linear(a, m_.weight, m_.bias))
    gn = nn.GroupNorm(8, 32).cuda()
    with torch.no_grad():
        gn.weight.uniform_(0.5, 1.5)
        gn.bias.uniform_(-0.5, 0.5)
    _check(gn, [torch.randn(2, 32, 9, 7)], lambda a: LF.group_norm(gn, a), lambda m_, a: m_(a))
    _check(gn, [torch.randn(2, 32, 63)], lambda a: LF.group_norm(gn, a, silu=True), lambda m_, a: F.silu(m_(a)))
    seq = nn.Sequential(nn.SiLU(), lin)
    _check(lin, [torch.randn(3, 24)], lambda a: LF.call(seq, a), lambda m_, a: m_(F.silu(a)))


@pytest.mark.parametrize("cross", [False, True])
def test_mha_leaf(cross):
    from sdmi import leaf as LF
    torch.manual_seed(2)
    m = nn.MultiheadAttention(64, 4, batch_first=True).cuda()
    q = torch.randn(2, 50, 64)
    if cross:
        kv = torch.randn(2, 13, 64)
        _check(m, [q, kv], lambda a, c: LF.call(m, a, c, c)[0], lambda m_, a, c: m_(a, c, c)[0])
    else:
        _check(m, [q], lambda a: LF.call(m, a, a, a)[0], lambda m_, a: m_(a, a, a)[0])


def test_down_block_standalone_vs_oracle():
    """DownBlock(x, t_emb, context) on its own (blocks.py:111-146) against the oracle's resnet / attention."""
    from models.blocks import DownBlock
    torch.manual_seed(3)
    blk = DownBlock(32, 64, 128, down_sample=True, num_heads=4, num_layers=2, attn=True, norm_channels=16,
                    cross_attn=True, context_dim=48).cuda()
    sd = {"b." + k: v.detach().cpu() for k, v in blk.state_dict().items()}
    x = torch.randn(2, 32, 16, 16)
    temb = torch.randn(2, 128)
    ctx = torch.randn(2, 11, 48)
    y = blk(x.cuda(), temb.cuda(), ctx.cuda())
    leaves = {k: v.clone().requires_grad_(True) for k, v in sd.items()}
    out = x
    for i in range(2):
        out = O.resnet(leaves, "b", i, out, temb, 16)
        out = O.self_attn(leaves, "b", i, out, 16, 4)
        out = O.cross_attn(leaves, "b", i, out, ctx, 16, 4)
    ref = O.conv(leaves, "b.down_sample_conv", out, stride=2, padding=1)
    assert rel(y.detach(), ref.detach()) <= 2e-2
    g = torch.randn(ref.shape, generator=torch.Generator().manual_seed(4))
    y.backward(g.cuda())
    ref.backward(g)
    for k, p in blk.named_parameters():
        r = leaves["b." + k].grad
        if r is not None and r.norm() > 1e-6:
            assert cos(p.grad, r) >= 0.99, k


class _SwappedConv(nn.Conv2d):
    calls = 0

    def forward(self, x):
        _SwappedConv.calls += 1
        return F.conv2d(x, self.weight, self.bias, self.stride, self.padding)


class _SwappedLinear(nn.Linear):
    calls = 0

    def forward(self, x):
        _SwappedLinear.calls += 1
        return F.linear(x, self.weight, self.bias)


def _swap_like_cim(model):
    """ProgressiveTrain.convert_to_layers (progressive_qn_train.py:576-651): exact nn.Conv2d / nn.Linear leaves are
    replaced by new layer objects that take over the Parameters (new.weight = module.weight)."""
    n = 0
    for name, mod in list(model.named_modules()):
        for cname, child in list(mod.named_children()):
            if type(child) is nn.Conv2d:
                new = _SwappedConv(child.in_channels, child.out_channels, child.kernel_size, child.stride,
                                   child.padding, bias=child.bias is not None).to(child.weight.device)
            elif type(child) is nn.Linear:
                new = _SwappedLinear(child.in_features, child.out_features, bias=child.bias is not None
                                     ).to(child.weight.device)
            else:
                continue
            new.weight = child.weight
            if child.bias is not None:
                new.bias = child.bias
            setattr(mod, cname, new)
            n += 1
    return n


def test_cond_unet_with_swapped_layers_vs_oracle():
    import models.unet_cond_base as mc
    torch.manual_seed(5)
    sd = O.deterministic_state(O.unet_param_shapes(SMALL_COND, base="cond"), 5)
    model = mc.Unet(4, SMALL_COND).cuda()
    model.load_state_dict(sd)
    g = torch.Generator().manual_seed(6)
    x = torch.randn(2, 4, 32, 32, generator=g)
    t = torch.randint(0, 1000, (2,), generator=g)
    cmap = torch.randint(0, 19, (2, 64, 64), generator=g)
    mask = F.one_hot(cmap, 19).movedim(-1, 1)[:, 1:].float()
    text = torch.randn(2, 77, SMALL_COND["condition_config"]["text_condition_config"]["text_embed_dim"], generator=g)
    half = len([m for m in model.modules() if type(m) in (nn.Conv2d, nn.Linear)]) // 2
    # swap only some leaves: the model mixes HIP leaves and swapped ones
    for i, (name, mod) in enumerate([(n, m) for n, m in model.named_modules() if type(m) in (nn.Conv2d, nn.Linear)]):
        if i % 2 == 0:
            parent = model.get_submodule(name.rsplit(".", 1)[0]) if "." in name else model
            cname = name.rsplit(".", 1)[-1]
            if type(mod) is nn.Conv2d:
                new = _SwappedConv(mod.in_channels, mod.out_channels, mod.kernel_size, mod.stride, mod.padding,
                                   bias=mod.bias is not None).cuda()
            else:
                new = _SwappedLinear(mod.in_features, mod.out_features, bias=mod.bias is not None).cuda()
            new.weight = mod.weight
            if mod.bias is not None:
                new.bias = mod.bias
            setattr(parent, cname, new)
    assert half > 0
    _SwappedConv.calls = _SwappedLinear.calls = 0
    out = model(x.cuda(), t.cuda(), {"image": mask.cuda(), "text": text.cuda()})
    assert _SwappedConv.calls > 0 and _SwappedLinear.calls > 0
    leaves = {k: v.clone().requires_grad_(True) for k, v in sd.items()}
    ref = O.unet_forward(leaves, SMALL_COND, x, t, {"image": mask, "text": text})
    assert rel(out.detach(), ref.detach()) <= 3e-2
    noise = torch.randn(x.shape, generator=torch.Generator().manual_seed(7))
    F.mse_loss(out, noise.cuda()).backward()
    F.mse_loss(ref, noise).backward()
    worst = min((cos(p.grad, leaves[k].grad), k) for k, p in model.named_parameters()
                if leaves[k].grad is not None and leaves[k].grad.norm() > 1e-6)
    assert worst[0] >= 0.99, worst


def test_vqvae_with_swapped_layers_vs_reference():
    from models.vqvae import VQVAE
    f = load_file(os.path.join(G, "vqvae_small.safetensors"))
    sd = O.deterministic_state(VO.vqvae_param_shapes(SMALL_VQVAE), seed=9)
    model = VQVAE(3, SMALL_VQVAE).cuda()
    model.load_state_dict(sd)
    assert _swap_like_cim(model) > 10
    assert model._leaf()
    _SwappedConv.calls = 0
    with torch.no_grad():
        zq, losses, idx = model._leaf_encode(f["x"].cuda())
        out = model.decode(f["zq"].cuda())
    assert _SwappedConv.calls > 0
    assert (idx.cpu() == f["indices"]).float().mean().item() >= 0.8
    assert rel(out, f["out"]) <= 3e-2
    # training through the swapped model: recon + codebook + commitment, every parameter gets a finite gradient
    x = f["x"].cuda()
    out, z, ql = model(x)
    (F.mse_loss(out, x) + ql["codebook_loss"] + 0.2 * ql["commitment_loss"]).backward()
    for k, p in model.named_parameters():
        assert p.grad is not None and torch.isfinite(p.grad).all(), k
    assert model.encoder_conv_in.weight.grad.norm() > 0 and model.embedding.weight.grad.norm() > 0


@pytest.mark.parametrize("swap", [False, True])
def test_dit_leaf_path_vs_oracle(swap):
    """The DIT forced onto the leaf path (sdmi_leaf_path) or with its nn.Linear / nn.Conv2d leaves swapped:
    TransformerLayer / Attention / CustomMultiheadAttention / PatchEmbedding forwards (transformer_layer.py:80-106,
    attention.py:33-78, multihead_attention.py:41-80, patch_embed.py:75-96) against the oracle and the reference
    fixture (text + image conditioning)."""
    from models.transformer import DIT
    from oracle import dit_oracle as DO
    from tests.golden.configs import SMALL_DIT
    f = load_file(os.path.join(G, "dit_small.safetensors"))
    sd = O.deterministic_state(DO.dit_param_shapes(SMALL_DIT), 4)
    model = DIT(4, SMALL_DIT).cuda()
    model.load_state_dict(sd)
    if swap:
        assert _swap_like_cim(model) > 10
    else:
        model.sdmi_leaf_path = True
    c = {"text": f["text"], "image": F.one_hot(f["classmap"].long(), 19).movedim(-1, 1)[:, 1:].float()}
    _SwappedLinear.calls = 0
    out = model(f["x"].cuda(), f["t"].cuda(), {k: v.cuda() for k, v in c.items()})
    assert (_SwappedLinear.calls > 0) == swap
    leaves = {k: v.clone().requires_grad_(True) for k, v in sd.items()}
    ref = DO.dit_forward(leaves, SMALL_DIT, f["x"], f["t"], c)
    assert ((out.detach().cpu() - ref.detach()) ** 2).mean().item() <= 1e-4
    assert ((out.detach().cpu() - f["out"]) ** 2).mean().item() <= 1e-4
    F.mse_loss(out, f["noise"].cuda()).backward()
    F.mse_loss(ref, f["noise"]).backward()
    worst = min((cos(p.grad, leaves[k].grad), k) for k, p in model.named_parameters()
                if leaves[k].grad is not None and leaves[k].grad.norm() > 1e-6)
    assert worst[0] >= 0.99, worst


def test_linear_leaf_ragged_features():
    """Linear with in / out features that are not multiples of 8 (the DiT patch embedding: 2*2*(4+3) = 28)."""
    from sdmi import leaf as LF
    torch.manual_seed(8)
    lin = nn.Linear(28, 13).cuda()
    _check(lin, [torch.randn(2, 9, 28)], lambda a: LF.linear(lin, a), lambda m_, a: F.linear(a, m_.weight, m_.bias))
