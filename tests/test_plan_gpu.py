"""Launch-plan replay (sdmi.plan.StepPlan) reproduces eager training steps bit for bit: the recorded native
calls re-issued with the same pointers / streams / order on fresh per-step inputs (static buffers) give the same
parameters, Adam moments and loss as issuing every step eagerly (all kernels are deterministic: no atomics)."""
import pytest
import torch

from oracle import sd_oracle as O
from oracle import dit_oracle as DO
from tests.golden.configs import SMALL_COND, SMALL_DIT

pytestmark = pytest.mark.gpu


def _inputs(step, B=2):
    g = torch.Generator().manual_seed(700 + step)
    x0 = torch.randn(B, 4, 32, 32, generator=g)
    noise = torch.randn(B, 4, 32, 32, generator=g)
    t = torch.randint(0, 1000, (B,), generator=g)
    text = torch.randn(B, 77, 64, generator=g)
    cmap = torch.randint(0, 19, (B, 64, 64), generator=g)
    mask = torch.nn.functional.one_hot(cmap, 19).movedim(-1, 1)[:, 1:].float()
    keep = (torch.rand(B, generator=g) > 0.3).float()
    return [v.cuda() for v in (x0, noise, t, text, mask, keep)]


@pytest.mark.parametrize("model", ["unet", "dit"])
def test_plan_replay_matches_eager(model):
    from sdmi.trainer import DDPMTrainer
    from sdmi.plan import StepPlan
    if model == "dit":
        sd = O.deterministic_state(DO.dit_param_shapes(SMALL_DIT), seed=2)
        mk = lambda: DDPMTrainer(SMALL_DIT, sd, "cuda", base="dit", lr=1e-3, ema_decay=None)  # noqa: E731
    else:
        sd = O.deterministic_state(O.unet_param_shapes(SMALL_COND), seed=2)
        mk = lambda: DDPMTrainer(SMALL_COND, sd, "cuda", lr=1e-3)  # noqa: E731
    eager, planned = mk(), mk()
    bufs = [torch.empty_like(v) for v in _inputs(0)]

    def run(tr):
        tr.step(*bufs[:5], mask_keep=bufs[5])

    steps = 4
    for s in range(steps):
        for b, v in zip(bufs, _inputs(s)):
            b.copy_(v)
        run(eager)
    torch.cuda.synchronize()
    for s in range(steps):
        for b, v in zip(bufs, _inputs(s)):
            b.copy_(v)
        if s == 0:
            plan = StepPlan(lambda: run(planned))
            assert len(plan) > 50
        else:
            plan.replay()
    torch.cuda.synchronize()
    assert torch.equal(eager.store.params, planned.store.params)
    assert torch.equal(eager.m, planned.m) and torch.equal(eager.v, planned.v)
    assert torch.equal(eager.state, planned.state)
    if eager.ema is not None:
        assert torch.equal(eager.ema, planned.ema)


@pytest.mark.parametrize("model", ["unet", "dit"])
def test_bf16_image_matches_full_repack(model, monkeypatch):
    """The optimizer writes a bf16 image of the flat parameters (sdmi_adam_ema_bf16) and the engine reads every
    identity-layout weight from it (PackPlan aliases): three steps bit-identical to packing every weight from the fp32
    masters (SDMI_SHADOW=0), and the aliases really are used."""
    from sdmi.trainer import DDPMTrainer
    if model == "dit":
        sd = O.deterministic_state(DO.dit_param_shapes(SMALL_DIT), seed=3)
        mk = lambda: DDPMTrainer(SMALL_DIT, sd, "cuda", base="dit", lr=1e-3, ema_decay=None)  # noqa: E731
    else:
        sd = O.deterministic_state(O.unet_param_shapes(SMALL_COND), seed=3)
        mk = lambda: DDPMTrainer(SMALL_COND, sd, "cuda", lr=1e-3)  # noqa: E731
    monkeypatch.setenv("SDMI_SHADOW", "1")
    img = mk()
    monkeypatch.setenv("SDMI_SHADOW", "0")
    full = mk()  # the default
    assert full.shadow is None and not full.engine.pack.alias
    assert img.shadow is not None and len(img.engine.pack.alias) >= 8, sorted(img.engine.pack.alias)
    for s in range(3):
        ins = _inputs(s)
        for tr in (img, full):
            tr.step(*ins[:5], mask_keep=ins[5])
    torch.cuda.synchronize()
    img.sync_optimizer()
    full.sync_optimizer()
    torch.cuda.synchronize()
    assert torch.equal(img.store.params, full.store.params)
    assert torch.equal(img.m, full.m) and torch.equal(img.state, full.state)
    # the image is the bf16 rounding of the masters
    assert torch.equal(img.shadow, img.store.params.to(torch.bfloat16))
    for name in img.engine.pack.alias:  # aliased views equal the packed copies of the fp32 masters
        assert torch.equal(img.engine.pack.view(name), full.engine.pack.view(name)), name


@pytest.mark.parametrize("model", ["unet", "dit"])
def test_norm_in_pieces_matches_one_pass(model, monkeypatch):
    """clip_grad_norm_'s sum of squares issued in pieces during the backward (sdmi.trainer.NormParts) gives the norm of
    the one-pass sdmi_clip_unscale (SDMI_NORM_PARTS=0) to fp32 rounding, and the same steps."""
    from sdmi.trainer import DDPMTrainer
    if model == "dit":
        sd = O.deterministic_state(DO.dit_param_shapes(SMALL_DIT), seed=4)
        mk = lambda: DDPMTrainer(SMALL_DIT, sd, "cuda", base="dit", lr=1e-3, ema_decay=None)  # noqa: E731
    else:
        sd = O.deterministic_state(O.unet_param_shapes(SMALL_COND), seed=4)
        mk = lambda: DDPMTrainer(SMALL_COND, sd, "cuda", lr=1e-3)  # noqa: E731
    monkeypatch.setenv("SDMI_NORM_PARTS", "1")
    parts = mk()
    monkeypatch.setenv("SDMI_NORM_PARTS", "0")
    one = mk()
    assert parts.norm_parts is not None and one.norm_parts is None
    parts.norm_parts.chunk = 1 << 16  # several pieces for the small model (the default is 64 MB)
    for s in range(3):
        ins = _inputs(s)
        for tr in (parts, one):
            tr.step(*ins[:5], mask_keep=ins[5])
        torch.cuda.synchronize()
        assert parts.norm_parts.used > parts.norm_parts._blocks(1 << 16)  # more than one piece
        a, b = parts.state[0].item(), one.state[0].item()
        assert abs(a - b) <= 1e-5 * b, (s, a, b)
    parts.sync_optimizer()
    one.sync_optimizer()
    torch.cuda.synchronize()
    assert torch.equal(parts.state[2:6], one.state[2:6])  # scale, growth tracker, step, skip flag
    d = (parts.store.params - one.store.params).abs().max().item()
    assert d <= 1e-6, d
