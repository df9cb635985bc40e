"""Captured DDPM sampling loop: the reference's sampler (tools/sample_ddpm_vqvae.py:29-52, and the conditional
tools/sample_ddpm_text_image_cond.py loop) -- T x [model(x_t, t) -> LinearNoiseScheduler.sample_prev_timestep] --
recorded ONCE as a native launch plan and replayed T times with no host work per step.

Everything a step needs lives on the device: the timestep t is an int64 device scalar read by the time-embedding
kernel and by sdmi_ddpm_prev, which decrements it after the step; the noise z comes from the Philox kernel
(sdmi_randn) keyed by (seed, device draw counter) that advances per replay; x_t is updated in place. The
reference instead moves t to the device, draws z with the host generator and syncs on `t == 0` every step
(scheduler/linear_noise_scheduler.py:66-72) and repacks nothing -- here the weights are packed once per loop
(sdmi.module_glue version check)."""
import ctypes

import torch

from . import _lib
from . import kernels as K
from .plan import StepPlan


class DDPMSampleLoop:
    def __init__(self, model, scheduler, shape, cond_input=None, seed=0):
        """model: a drop-in denoiser module (models.unet_cond_base.Unet / unet_base.Unet / transformer.DIT) already
        on the GPU; scheduler: scheduler.linear_noise_scheduler.LinearNoiseScheduler; shape: (B, C, H, W) latents;
        cond_input: the model's condition dict (text / image / class), fixed for the whole loop."""
        dev = next(model.parameters()).device
        if dev.type != "cuda":
            raise RuntimeError("the sampling loop runs on the MI355X HIP path only (move the model to cuda)")
        self.dev = dev
        holder = model._sdmi
        self.eng = holder.ensure(dev)
        holder.refresh([p for _, p in model.named_parameters()])
        self.T = scheduler.num_timesteps
        self.tab = scheduler.tables(dev)
        B, C, H, W = shape
        self.shape = (B, C, H, W)
        self.xt = torch.empty(shape, dtype=torch.float32, device=dev)
        self.z = torch.empty_like(self.xt)
        self.x0 = torch.empty_like(self.xt)
        self.eps = None  # the model output of the last step (a buffer of the recorded plan)
        self.t = torch.zeros(1, dtype=torch.int64, device=dev)
        self.offset = torch.zeros(1, dtype=torch.int64, device=dev)  # Philox draw counter (uint64 bits)
        self.seed = int(seed)
        c = cond_input or {}
        self.text, self.mask, self.klass = c.get("text"), c.get("image"), c.get("class")
        self.plan = None

    def _step(self):
        B, C, H, W = self.shape
        pred, _ = self.eng.forward(self.xt, self.t, self.text, self.mask, need_backward=False, klass=self.klass)
        self.eps = self.eng.pred_to_nchw(pred, B, H, W)
        L = _lib.lib()
        n = self.xt.numel()
        _lib.check(L.sdmi_randn(self.z.data_ptr(), n, ctypes.c_ulonglong(self.seed), self.offset.data_ptr(), 1,
                                K._stream()), "sdmi_randn")
        tab = self.tab
        _lib.check(L.sdmi_ddpm_prev(self.xt.data_ptr(), self.eps.data_ptr(), self.z.data_ptr(), n, self.t.data_ptr(),
                                    tab["betas"].data_ptr(), tab["alphas"].data_ptr(), tab["alpha_cum_prod"].data_ptr(),
                                    tab["sqrt_one_minus_alpha_cum_prod"].data_ptr(), self.xt.data_ptr(),
                                    self.x0.data_ptr(), 1, K._stream()), "sdmi_ddpm_prev")

    def reset(self, x_T, t_start=None, draw=0):
        """Start a loop from x_T at timestep t_start (default T - 1) with the noise draw counter at `draw`."""
        self.xt.copy_(x_T)
        self.t.fill_(self.T - 1 if t_start is None else int(t_start))
        self.offset.fill_(int(draw))

    def run(self, x_T, steps=None, captured=True, t_start=None):
        """`steps` (default T) reverse steps from x_T; returns (x_{t_end}, x0 prediction of the last step).
        captured=False issues every step eagerly (the stepwise reference loop, same kernels and order)."""
        self.reset(x_T, t_start)
        steps = self.T if steps is None else int(steps)
        for i in range(steps):
            if not captured:
                self._step()
            elif self.plan is None:  # the first step is recorded while it runs
                self.plan = StepPlan(self._step, self.dev)
            else:
                self.plan.replay()
        return self.xt, self.x0
