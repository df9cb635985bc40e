"""GPU sampling-step kernels (csrc/sampler.hip) against the reference's own outputs: bit-exact.

sdmi_ddpm_prev uses the reference's fp32 tables (from the golden fixture: torch-CPU table rounding differs by
<= 1 ulp between host CPUs, see test_unet_gpu.test_scheduler_add_noise_bit_exact), reads the timestep from device
memory and must reproduce x_{t-1} and x0 of LinearNoiseScheduler.sample_prev_timestep bit for bit for the same z;
the DDIM / DDPM sampler steps likewise against DDIMSampler / DDPMSampler.sample_one_step with a fixed-output model."""
import os

import pytest
import torch
from safetensors.torch import load_file

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def fx(name):
    return load_file(os.path.join(G, name + ".safetensors"))


@pytest.mark.parametrize("name,b0,b1", [("cond", 0.00085, 0.012), ("uncond", 0.0015, 0.0195)])
def test_ddpm_prev_bit_exact(name, b0, b1):
    from scheduler.linear_noise_scheduler import LinearNoiseScheduler
    f = fx(f"scheduler_{name}")
    s = LinearNoiseScheduler(1000, b0, b1)
    for k in ("betas", "alphas", "alpha_cum_prod", "sqrt_alpha_cum_prod", "sqrt_one_minus_alpha_cum_prod"):
        setattr(s, k, f[k])
    s._dev = {}
    xt, eps, z = f["xt"].cuda(), (f["eps"] * 0.9).cuda(), f["z"].cuda()
    for t, key in ((500, "500"), (0, "0")):
        prev, x0 = s.sample_prev_timestep(xt, eps, t, z=z)
        assert torch.equal(prev.cpu(), f[f"prev_{key}"]), t
        assert torch.equal(x0.cpu(), f[f"x0hat_{key}"]), t
    # device-resident timestep with in-kernel decrement (capturable sampling loop)
    t_dev = torch.tensor([500], dtype=torch.int64, device="cuda")
    prev, x0 = s.sample_prev_timestep(xt, eps, t_dev, z=z, decrement_t=True)
    torch.cuda.synchronize()
    assert torch.equal(prev.cpu(), f["prev_500"]) and t_dev.item() == 499


def test_ddim_and_ddpm_sampler_steps_bit_exact():
    from scheduler.linear_noise_scheduler import DDIMSampler, DDPMSampler
    f = fx("samplers")
    eps = f["eps"].cuda()

    class Fixed(torch.nn.Module):
        def forward(self, *a, **k):
            return eps

    x, noise = f["x"].cuda(), f["noise"].cuda()
    ddim = DDIMSampler(Fixed(), beta=(0.00085, 0.012), T=1000)
    ddim.alpha_t_bar = f["ddim_alpha_t_bar"]  # the reference's own table (host-CPU cumprod rounding varies)
    ddim.cond_input = None
    for eta in (0.0, 1.0):
        for (t, tp) in ((801, 760), (11, 1), (1, 0)):
            out = ddim.sample_one_step(x, t, tp, eta, noise=noise)
            assert torch.equal(out.cpu(), f[f"ddim_eta{eta:g}_{t}_{tp}"]), (eta, t, tp)
    ddpm = DDPMSampler(Fixed(), beta=(0.0001, 0.02), T=1000)
    for k in ("coeff_1", "coeff_2", "posterior_variance"):
        getattr(ddpm, k).copy_(f[f"ddpm_{k}"])
    for t in (999, 500, 0):
        out = ddpm.sample_one_step(x, t, z=noise)
        assert torch.equal(out.cpu(), f[f"ddpm_{t}"]), t
