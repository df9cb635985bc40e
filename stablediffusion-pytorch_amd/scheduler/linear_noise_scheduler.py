"""Drop-in scheduler module (reference scheduler/linear_noise_scheduler.py): LinearNoiseScheduler (:8-78),
DDPMSampler (:93-150) and DDIMSampler (:153-232).

The beta/alpha tables are built on the host exactly as the reference builds them (fp32 torch on
CPU: linspace of sqrt-betas squared, cumprod) so they are bit-identical; per-device copies are cached
once instead of being re-uploaded on every call (reference :37-38). add_noise runs as one HIP kernel
(sdmi_add_noise) with the same fp32 mul/mul/add order, so x_t is bit-identical to the reference for
the same (x0, noise, t)."""
import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from sdmi import _lib
from sdmi import kernels as K
from sdmi import plan


def _require_cuda(t, what):
    if not t.is_cuda:
        raise RuntimeError(f"sdmi {what} runs on the HIP path only (cuda tensors)")
    _lib.lib()


class LinearNoiseScheduler:
    def __init__(self, num_timesteps, beta_start, beta_end):
        self.num_timesteps = num_timesteps
        self.beta_start = beta_start
        self.beta_end = beta_end
        self.betas = torch.linspace(beta_start ** 0.5, beta_end ** 0.5, num_timesteps) ** 2
        self.alphas = 1. - self.betas
        self.alpha_cum_prod = torch.cumprod(self.alphas, dim=0)
        self.sqrt_alpha_cum_prod = torch.sqrt(self.alpha_cum_prod)
        self.sqrt_one_minus_alpha_cum_prod = torch.sqrt(1 - self.alpha_cum_prod)
        self._dev = {}

    def tables(self, device):
        key = str(device)
        if key not in self._dev:
            self._dev[key] = {n: getattr(self, n).to(device) for n in
                              ("betas", "alphas", "alpha_cum_prod", "sqrt_alpha_cum_prod",
                               "sqrt_one_minus_alpha_cum_prod")}
        return self._dev[key]

    def add_noise(self, original, noise, t):
        """x_t = sqrt(abar_t) x0 + sqrt(1 - abar_t) eps, t of shape (B,) (reference :26-48)."""
        if not original.is_cuda:
            raise RuntimeError("sdmi LinearNoiseScheduler.add_noise runs on the HIP path only (cuda tensors)")
        tab = self.tables(original.device)
        x0 = plan.as_operand(original)
        eps = plan.as_operand(noise)
        tt = plan.timesteps(t, original.device)
        if tt.numel() != x0.shape[0]:
            raise ValueError("t must have one timestep per sample")
        out = torch.empty_like(x0)
        return K.add_noise(x0, eps, tt, tab["sqrt_alpha_cum_prod"], tab["sqrt_one_minus_alpha_cum_prod"], out)

    def sample_prev_timestep(self, xt, noise_pred, t, z=None, out=None, decrement_t=False):
        """DDPM reverse step (reference :50-78) as ONE fused kernel (sdmi_ddpm_prev), bit-identical to the
        reference for the same z. t: int, 0-d / (1,) tensor (host or device; a device int64 tensor is read by the
        kernel itself, no host sync). z: None draws torch.randn(xt.shape) on the CPU generator exactly like the
        reference (:72) for t > 0 -- pass a device tensor to keep sampling on the GPU. out: optional preallocated
        (x_prev, x0) buffers; decrement_t: the kernel decrements the device timestep after the step (a captured
        sampling step can then be replayed T times)."""
        _require_cuda(xt, "LinearNoiseScheduler.sample_prev_timestep")
        tab = self.tables(xt.device)
        x = plan.as_operand(xt)
        e = plan.as_operand(noise_pred)
        if isinstance(t, torch.Tensor) and t.is_cuda and t.dtype == torch.int64:
            t_dev = t.reshape(-1)[:1]
            if z is None:  # t unknown on the host: always draw (unused by the kernel at t == 0)
                z = torch.randn(xt.shape).to(xt.device)
        else:
            ti = int(t)
            t_dev = torch.tensor([ti], dtype=torch.int64, device=xt.device)
            if z is None and ti > 0:
                z = torch.randn(xt.shape).to(xt.device)
        prev, x0 = out if out is not None else (torch.empty_like(x), torch.empty_like(x))
        zz = plan.as_operand(z) if z is not None else None
        _lib.check(_lib.lib().sdmi_ddpm_prev(x.data_ptr(), e.data_ptr(), K._p(zz), x.numel(), t_dev.data_ptr(),
                                             tab["betas"].data_ptr(), tab["alphas"].data_ptr(),
                                             tab["alpha_cum_prod"].data_ptr(),
                                             tab["sqrt_one_minus_alpha_cum_prod"].data_ptr(), prev.data_ptr(),
                                             x0.data_ptr(), int(decrement_t), K._stream()), "sdmi_ddpm_prev")
        return prev, x0


def extract(v, i, shape):
    """reference :81-90: v[i] reshaped to (batch, 1, 1, ...)."""
    out = torch.gather(v, index=i, dim=0).to(device=i.device, dtype=torch.float32)
    return out.view([i.shape[0]] + [1] * (len(shape) - 1))


class DDPMSampler(nn.Module):
    """reference :93-150 (Alokia/diffusion-DDIM-pytorch): linear beta schedule linspace(beta), coefficients
    precomputed as buffers; each step is the model forward plus one fused elementwise kernel."""

    def __init__(self, model, beta, T):
        super().__init__()
        self.model = model
        self.T = T
        self.register_buffer("beta_t", torch.linspace(*beta, T, dtype=torch.float32))
        alpha_t = 1.0 - self.beta_t
        alpha_t_bar = torch.cumprod(alpha_t, dim=0)
        alpha_t_bar_prev = F.pad(alpha_t_bar[:-1], (1, 0), value=1.0)
        self.register_buffer("coeff_1", torch.sqrt(1.0 / alpha_t))
        self.register_buffer("coeff_2", self.coeff_1 * (1.0 - alpha_t) / torch.sqrt(1.0 - alpha_t_bar))
        self.register_buffer("posterior_variance", self.beta_t * (1.0 - alpha_t_bar_prev) / (1.0 - alpha_t_bar))

    @torch.no_grad()
    def sample_one_step(self, x_t, time_step, z=None):
        _require_cuda(x_t, "DDPMSampler")
        t = torch.full((x_t.shape[0],), time_step, device=x_t.device, dtype=torch.long)
        eps = self.model(x_t, t).float().contiguous()
        ts = int(time_step)
        c1, c2 = self.coeff_1[ts].item(), self.coeff_2[ts].item()
        var = self.posterior_variance[ts].item()  # square-rooted in the kernel (correctly rounded)
        if ts > 0 and z is None:
            z = torch.randn_like(x_t)
        x = x_t.float().contiguous()
        out = torch.empty_like(x)
        zz = z.float().contiguous() if ts > 0 else None
        _lib.check(_lib.lib().sdmi_affine_step(x.data_ptr(), eps.data_ptr(), K._p(zz), x.numel(), c1, c2, var,
                                               out.data_ptr(), K._stream()), "sdmi_affine_step")
        if torch.isnan(out).int().sum() != 0:
            raise ValueError("nan in tensor!")
        return out

    @torch.no_grad()
    def forward(self, x_t, only_return_x_0=True, interval=1, **kwargs):
        x = [x_t]
        for time_step in reversed(range(self.T)):
            x_t = self.sample_one_step(x_t, time_step)
            if not only_return_x_0 and ((self.T - time_step) % interval == 0 or time_step == 0):
                x.append(torch.clip(x_t, -1.0, 1.0))
        return x_t if only_return_x_0 else torch.stack(x, dim=1)


class DDIMSampler(nn.Module):
    """reference :153-232: linspace(beta) schedule, "linear" / "quadratic" step selection (+1 offset), eta; each
    step is the model forward with the sampler's cond_input plus one fused elementwise kernel."""

    def __init__(self, model, beta, T):
        super().__init__()
        self.model = model
        self.T = T
        beta_t = torch.linspace(*beta, T, dtype=torch.float32)
        self.alpha_t_bar = torch.cumprod(1.0 - beta_t, dim=0)

    @torch.no_grad()
    def sample_one_step(self, x_t, time_step, prev_time_step, eta, noise=None):
        _require_cuda(x_t, "DDIMSampler")
        t = torch.full((x_t.shape[0],), int(time_step), device=x_t.device, dtype=torch.long)
        eps = self.model(x_t, t, self.cond_input).float().contiguous()
        if noise is None:
            noise = torch.randn_like(x_t)  # drawn every step, as the reference does (:171)
        x = x_t.float().contiguous()
        out = torch.empty_like(x)
        at = self.alpha_t_bar[int(time_step)].item()
        ap = self.alpha_t_bar[int(prev_time_step)].item()
        _lib.check(_lib.lib().sdmi_ddim_prev(x.data_ptr(), eps.data_ptr(), noise.float().contiguous().data_ptr(),
                                             x.numel(), at, ap, float(eta), out.data_ptr(), K._stream()),
                   "sdmi_ddim_prev")
        return out

    @staticmethod
    def time_steps(T, steps, method="linear"):
        if method == "linear":
            ts = np.asarray(list(range(0, T, T // steps)))
        elif method == "quadratic":
            ts = (np.linspace(0, np.sqrt(T * 0.8), steps) ** 2).astype(np.int32)
        else:
            raise NotImplementedError(f"sampling method {method} is not implemented!")
        ts = ts + 1
        return ts, np.concatenate([[0], ts[:-1]])

    @torch.no_grad()
    def forward(self, x_t, cond_input, uncond_input, steps=1, method="linear", eta=0.0, only_return_x_0=True,
                interval=1, captured=True, seed=None):
        """captured (default): a drop-in denoiser on the fused engine samples through sdmi.sampling.DDIMSampleLoop --
        the loop recorded once and replayed with device timestep tables and device noise (Philox) -- when only x_0 is
        returned; otherwise (intermediates, foreign models) every step is issued eagerly with torch.randn_like noise as
        the reference does (:200). seed=None (default): every call draws fresh noise, its Philox stream chosen by
        torch's default generator (as the reference's randn_like is, so torch.manual_seed makes a call repeatable);
        an explicit seed makes every call with that seed repeat the same noise."""
        self.cond_input = cond_input
        self.uncond_input = uncond_input
        if captured and only_return_x_0 and hasattr(self.model, "_sdmi"):
            from sdmi.module_glue import engine_path_ok
            from sdmi.sampling import DDIMSampleLoop
            if engine_path_ok(self.model):
                cond_key = tuple(sorted((k, v.data_ptr(), tuple(v.shape)) for k, v in (cond_input or {}).items()
                                        if isinstance(v, torch.Tensor)))
                # the parameters' identity is part of the key: replaced (not updated-in-place) weights rebuild the loop
                params = tuple(p.data_ptr() for p in self.model.parameters())
                key = (tuple(x_t.shape), steps, method, float(eta), -1 if seed is None else int(seed), cond_key,
                       hash(params))
                loop = getattr(self, "_loop", None)
                if loop is None or self._loop_key != key:
                    loop = DDIMSampleLoop(self.model, self.alpha_t_bar, tuple(x_t.shape), cond_input, steps=steps,
                                          method=method, eta=eta, seed=0 if seed is None else seed)
                    self._loop, self._loop_key = loop, key
                draw = loop.fresh_draw() if seed is None else 0
                return loop.run(x_t.float(), draw=draw).clone()
        ts, tp = self.time_steps(self.T, steps, method)
        x = [x_t]
        for i in reversed(range(0, steps)):
            x_t = self.sample_one_step(x_t, ts[i], tp[i], eta)
            if not only_return_x_0 and ((steps - i) % interval == 0 or i == 0):
                x.append(torch.clip(x_t, -1.0, 1.0))
        return x_t if only_return_x_0 else torch.stack(x, dim=1)
