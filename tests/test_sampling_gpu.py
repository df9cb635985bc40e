"""Captured DDPM sampling loop (sdmi.sampling.DDPMSampleLoop; reference tools/sample_ddpm_vqvae.py:29-52):
* the recorded-and-replayed loop is bit-identical to issuing every step eagerly (same kernels, device timestep,
  device noise);
* one step equals the reference arithmetic (oracle sample_prev_timestep, pinned bit-exact to the reference) on the
  model output and noise the step used (to a few ulp: host-CPU torch rounding), and the device timestep counts down;
* the Philox noise is standard normal and fresh per replay."""
import pytest
import torch

from oracle import sd_oracle as O
from tests.golden.configs import SMALL_COND, SMALL_UNCOND

pytestmark = pytest.mark.gpu


def one_hot(cmap, n=18):
    return torch.nn.functional.one_hot(cmap.long().clamp(0, n), n + 1).movedim(-1, 1)[:, 1:].float()


def _model(cond, seed=3):
    import models.unet_cond_base as mc
    import models.unet_base as mu
    cfg = SMALL_COND if cond else SMALL_UNCOND
    m = (mc.Unet if cond else mu.Unet)(4, cfg)
    m.load_state_dict(O.deterministic_state(O.unet_param_shapes(cfg, base="cond" if cond else "uncond"), seed))
    return m.cuda().eval()


@pytest.mark.parametrize("issue", ["graph", "plan"])
@pytest.mark.parametrize("cond", [False, True])
def test_captured_loop_matches_stepwise(cond, issue, monkeypatch):
    monkeypatch.setenv("SDMI_SAMPLE_ISSUE", issue)  # one hipGraph per step, or the native launch plan
    from sdmi.sampling import DDPMSampleLoop
    from scheduler.linear_noise_scheduler import LinearNoiseScheduler
    model = _model(cond)
    g = torch.Generator().manual_seed(9)
    B = 2
    c = None
    if cond:
        c = {"text": torch.randn(B, 77, 64, generator=g).cuda(),
             "image": one_hot(torch.randint(0, 19, (B, 64, 64), generator=g)).cuda()}
    xT = torch.randn(B, 4, 32, 32, generator=g).cuda()
    sched = LinearNoiseScheduler(1000, 0.00085, 0.012)
    cap = DDPMSampleLoop(model, sched, (B, 4, 32, 32), cond_input=c, seed=11)
    assert cap.issue == issue
    xa, x0a = (v.clone() for v in cap.run(xT, steps=6, captured=True))
    assert cap.t.item() == 1000 - 1 - 6
    eag = DDPMSampleLoop(model, sched, (B, 4, 32, 32), cond_input=c, seed=11)
    xb, x0b = eag.run(xT, steps=6, captured=False)
    torch.cuda.synchronize()
    assert torch.equal(xa, xb) and torch.equal(x0a, x0b)
    # a second captured run from the same start replays the recorded graph / plan: same result again
    xc, _ = cap.run(xT, steps=6, captured=True)
    assert torch.equal(xc, xa)
    if cond:  # the loop reads the context branch from its per-run cache: bitwise the module's own (uncached) forward
        one = DDPMSampleLoop(model, sched, (B, 4, 32, 32), cond_input=c, seed=11)
        one.run(xT, steps=1, captured=False)
        assert one.ctx_cache is not None
        with torch.no_grad():
            eps = model(xT, torch.tensor([999]).cuda(), c)
        assert torch.equal(eps, one.eps)


def test_one_step_matches_reference_arithmetic():
    from sdmi.sampling import DDPMSampleLoop
    from scheduler.linear_noise_scheduler import LinearNoiseScheduler
    model = _model(False)
    xT = torch.randn(2, 4, 32, 32, generator=torch.Generator().manual_seed(4)).cuda()
    sched = LinearNoiseScheduler(1000, 0.0015, 0.0195)
    loop = DDPMSampleLoop(model, sched, (2, 4, 32, 32), seed=2)
    for t0 in (999, 0):
        x, x0 = loop.run(xT, steps=1, captured=False, t_start=t0)
        torch.cuda.synchronize()
        ref_tab = O.SchedulerTables(1000, 0.0015, 0.0195)  # built on this host exactly like the module's tables
        prev, x0r = ref_tab.sample_prev_timestep(xT.cpu(), loop.eps.cpu(), t0, z=loop.z.cpu())
        # within a few ulp of the inputs' scale: this host's vectorised torch-CPU pow / sqrt / division rounding
        # differs between host CPUs (the kernel itself is pinned bit-exact to the reference's own outputs in
        # test_sampler_gpu.py)
        for a, b in ((x.cpu(), prev), (x0.cpu(), x0r)):
            tol = 4 * torch.finfo(torch.float32).eps * (b.abs() + xT.cpu().abs() + loop.eps.cpu().abs())
            assert ((a - b).abs() <= tol).all(), (t0, (a - b).abs().max().item())
        # the model output is the module's forward at t0 (the loop's eps buffer)
        with torch.no_grad():
            eps = model(xT, torch.tensor([t0]).cuda())
        assert torch.equal(eps, loop.eps)


def test_device_noise_is_standard_normal_and_fresh():
    from sdmi import _lib, kernels as K
    import ctypes
    n = 1 << 20
    z1 = torch.empty(n, device="cuda")
    z2 = torch.empty(n, device="cuda")
    off = torch.zeros(1, dtype=torch.int64, device="cuda")
    L = _lib.lib()
    _lib.check(L.sdmi_randn(z1.data_ptr(), n, ctypes.c_ulonglong(7), off.data_ptr(), 1, K._stream()), "randn")
    _lib.check(L.sdmi_randn(z2.data_ptr(), n, ctypes.c_ulonglong(7), off.data_ptr(), 1, K._stream()), "randn")
    torch.cuda.synchronize()
    assert off.item() == 2
    for z in (z1, z2):
        assert abs(z.mean().item()) < 5e-3 and abs(z.std().item() - 1) < 5e-3
        assert abs((z ** 4).mean().item() - 3) < 5e-2  # Gaussian kurtosis
    assert (z1 == z2).float().mean().item() < 1e-4
    off.zero_()
    _lib.check(L.sdmi_randn(z2.data_ptr(), n, ctypes.c_ulonglong(7), off.data_ptr(), 0, K._stream()), "randn")
    torch.cuda.synchronize()
    assert torch.equal(z1, z2) and off.item() == 0


@pytest.mark.parametrize("issue", ["graph", "plan"])
@pytest.mark.parametrize("method,eta", [("linear", 0.0), ("quadratic", 0.5)])
def test_captured_ddim_matches_stepwise(method, eta, issue, monkeypatch):
    """DDIMSampler.forward (reference scheduler/linear_noise_scheduler.py:209-256) as a recorded loop: device (t, t_prev)
    tables + device step index + device noise, bit-identical to issuing every step eagerly; the drop-in
    DDIMSampler.forward(captured=True) returns the same x_0; one step equals the module's eager sample_one_step
    (host-table alphas) on the same noise. Both captured issue modes (one hipGraph per step / the native plan)."""
    monkeypatch.setenv("SDMI_SAMPLE_ISSUE", issue)
    from sdmi.sampling import DDIMSampleLoop, ddim_time_steps
    from scheduler.linear_noise_scheduler import DDIMSampler
    model = _model(True)
    g = torch.Generator().manual_seed(12)
    B, steps = 2, 7
    c = {"text": torch.randn(B, 77, 64, generator=g).cuda(),
         "image": one_hot(torch.randint(0, 19, (B, 64, 64), generator=g)).cuda()}
    xT = torch.randn(B, 4, 32, 32, generator=g).cuda()
    sampler = DDIMSampler(model, (0.0001, 0.02), 1000)
    cap = DDIMSampleLoop(model, sampler.alpha_t_bar, (B, 4, 32, 32), c, steps=steps, method=method, eta=eta, seed=5)
    xa = cap.run(xT, captured=True).clone()
    ts, _ = ddim_time_steps(1000, steps, method)
    assert cap.idx.item() == 0 and cap.t.item() == int(ts[0])
    eag = DDIMSampleLoop(model, sampler.alpha_t_bar, (B, 4, 32, 32), c, steps=steps, method=method, eta=eta, seed=5)
    xb = eag.run(xT, captured=False)
    torch.cuda.synchronize()
    assert torch.isfinite(xa).all()
    assert torch.equal(xa, xb)
    assert torch.equal(cap.run(xT, captured=True), xa)  # replayed again from the same start
    xs = sampler(xT, c, None, steps=steps, method=method, eta=eta, seed=5)
    assert torch.equal(xs, xa)
    # one step vs the eager module step (sampler.sample_one_step: model forward + sdmi_ddim_prev with host alphas)
    one = DDIMSampleLoop(model, sampler.alpha_t_bar, (B, 4, 32, 32), c, steps=steps, method=method, eta=eta, seed=5)
    one.reset(xT)
    one._step()
    ts, tp = ddim_time_steps(1000, steps, method)
    ref = sampler.sample_one_step(xT, int(ts[steps - 1]), int(tp[steps - 1]), eta, noise=one.z)
    torch.cuda.synchronize()
    assert torch.equal(one.xt, ref)


def test_ddim_sampler_fresh_noise_per_call():
    """DDIMSampler.forward without a seed draws fresh noise per call like the reference's torch.randn_like (:200): two
    consecutive eta > 0 calls differ, torch.manual_seed makes a call repeatable, an explicit seed repeats its noise; a
    model whose parameters were replaced (not updated in place) rebuilds the captured loop."""
    from scheduler.linear_noise_scheduler import DDIMSampler
    model = _model(True)
    g = torch.Generator().manual_seed(13)
    B = 2
    c = {"text": torch.randn(B, 77, 64, generator=g).cuda(),
         "image": one_hot(torch.randint(0, 19, (B, 64, 64), generator=g)).cuda()}
    xT = torch.randn(B, 4, 32, 32, generator=g).cuda()
    sampler = DDIMSampler(model, (0.0001, 0.02), 1000)
    a = sampler(xT, c, None, steps=5, eta=1.0).clone()
    b = sampler(xT, c, None, steps=5, eta=1.0).clone()
    assert not torch.equal(a, b)
    torch.manual_seed(77)
    r1 = sampler(xT, c, None, steps=5, eta=1.0).clone()
    torch.manual_seed(77)
    r2 = sampler(xT, c, None, steps=5, eta=1.0).clone()
    assert torch.equal(r1, r2)
    s1 = sampler(xT, c, None, steps=5, eta=1.0, seed=4).clone()
    s2 = sampler(xT, c, None, steps=5, eta=1.0, seed=4).clone()
    assert torch.equal(s1, s2)
    loop = sampler._loop
    model.load_state_dict({k: v * 0.5 if k == "conv_out.weight" else v for k, v in model.state_dict().items()},
                          assign=True)
    s3 = sampler(xT, c, None, steps=5, eta=1.0, seed=4).clone()
    assert sampler._loop is not loop and not torch.equal(s3, s1)


def test_loop_refreshes_weights_and_honours_leaf_path():
    """A loop reused after a weight update written through `.data` (no version bump: the reference's EMA update)
    samples with the new weights; a model forced onto the leaf path is sampled stepwise through its own forward."""
    from sdmi.sampling import DDPMSampleLoop
    from scheduler.linear_noise_scheduler import LinearNoiseScheduler
    model = _model(False)
    xT = torch.randn(2, 4, 32, 32, generator=torch.Generator().manual_seed(6)).cuda()
    sched = LinearNoiseScheduler(1000, 0.0015, 0.0195)
    loop = DDPMSampleLoop(model, sched, (2, 4, 32, 32), seed=3)
    assert loop.fused
    a = loop.run(xT, steps=3)[0].clone()
    with torch.no_grad():
        model.conv_out.weight.data.mul_(0.5)
    b = loop.run(xT, steps=3)[0].clone()
    assert not torch.equal(a, b)
    fresh = DDPMSampleLoop(model, sched, (2, 4, 32, 32), seed=3)
    assert torch.equal(fresh.run(xT, steps=3)[0], b)
    model.sdmi_leaf_path = True
    leaf = DDPMSampleLoop(model, sched, (2, 4, 32, 32), seed=3)
    assert not leaf.fused
    c = leaf.run(xT, steps=3)[0]
    torch.cuda.synchronize()
    assert (c - b).abs().max().item() < 5e-2 * b.abs().max().item()
