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
def test_norm_in_pieces_matches_one_pass(model):
    """clip_grad_norm_'s sum of squares issued in pieces during the backward (sdmi.trainer.NormParts: fixed blocks at
    absolute flat offsets, watermarks rounded down to block boundaries) gives BITWISE the norm of the one-pass
    sdmi_clip_unscale over the whole buffer, hence bitwise the same steps (three steps, several pieces)."""
    from sdmi.trainer import DDPMTrainer
    if model == "dit":
        sd = O.deterministic_state(DO.dit_param_shapes(SMALL_DIT), seed=4)
        mk = lambda: DDPMTrainer(SMALL_DIT, sd, "cuda", base="dit", lr=1e-3, ema_decay=None)  # noqa: E731
    else:
        sd = O.deterministic_state(O.unet_param_shapes(SMALL_COND), seed=4)
        mk = lambda: DDPMTrainer(SMALL_COND, sd, "cuda", lr=1e-3)  # noqa: E731
    parts = mk()
    one = mk()
    one.norm_parts = None  # the whole-buffer pass (sdmi_clip_unscale)
    assert parts.norm_parts is not None
    blk = parts.norm_parts.blocks.blk
    parts.norm_parts.chunk = blk  # every finalised block range its own piece (the default is 64 MB)
    launches = []
    orig = parts.norm_parts.blocks.launch
    parts.norm_parts.blocks.launch = lambda g, lo, hi, st=None: (launches.append((lo, hi)), orig(g, lo, hi, st))
    for s in range(3):
        ins = _inputs(s)
        for tr in (parts, one):
            tr.step(*ins[:5], mask_keep=ins[5])
        torch.cuda.synchronize()
        assert parts.state[0].item() == one.state[0].item(), (s, parts.state[0].item(), one.state[0].item())
    assert len(launches) > 3, launches  # more than one piece per step
    parts.sync_optimizer()
    one.sync_optimizer()
    torch.cuda.synchronize()
    assert torch.equal(parts.state, one.state)
    assert torch.equal(parts.store.params, one.store.params)
