"""Drop-in LinearNoiseScheduler (reference scheduler/linear_noise_scheduler.py:8-78).

The beta/alpha tables are built on the host exactly as the reference builds them (fp32 torch on
CPU: linspace of sqrt-betas squared, cumprod) so they are bit-identical; per-device copies are cached
once instead of being re-uploaded on every call (reference :37-38). add_noise runs as one HIP kernel
(sdmi_add_noise) with the same fp32 mul/mul/add order, so x_t is bit-identical to the reference for
the same (x0, noise, t)."""
import torch

from sdmi import _lib
from sdmi import kernels as K


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
        x0 = original.float().contiguous()
        eps = noise.float().contiguous()
        tt = torch.as_tensor(t, device=original.device).long().reshape(-1).contiguous()
        if tt.numel() != x0.shape[0]:
            raise ValueError("t must have one timestep per sample")
        out = torch.empty_like(x0)
        return K.add_noise(x0, eps, tt, tab["sqrt_alpha_cum_prod"], tab["sqrt_one_minus_alpha_cum_prod"], out)

    def sample_prev_timestep(self, xt, noise_pred, t):
        """DDPM reverse step (reference :50-78), z drawn from the CPU generator as the reference does."""
        tab = self.tables(xt.device)
        t = int(t)
        x0 = (xt - tab["sqrt_one_minus_alpha_cum_prod"][t] * noise_pred) / torch.sqrt(tab["alpha_cum_prod"][t])
        x0 = torch.clamp(x0, -1., 1.)
        mean = xt - (tab["betas"][t] * noise_pred) / tab["sqrt_one_minus_alpha_cum_prod"][t]
        mean = mean / torch.sqrt(tab["alphas"][t])
        if t == 0:
            return mean, x0
        variance = (1 - tab["alpha_cum_prod"][t - 1]) / (1.0 - tab["alpha_cum_prod"][t]) * tab["betas"][t]
        z = torch.randn(xt.shape).to(xt.device)
        return mean + variance ** 0.5 * z, x0
