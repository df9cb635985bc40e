"""Captured sampling loops: the reference's samplers -- T x [model(x_t, t) -> LinearNoiseScheduler.sample_prev_timestep]
(tools/sample_ddpm_vqvae.py:29-52, tools/sample_ddpm_text_image_cond.py) and DDIMSampler.forward's
`steps` x [model(x_t, t, cond) -> DDIM update] (scheduler/linear_noise_scheduler.py:209-256) -- captured ONCE (as
one hipGraph per reverse step, default, or as sdmi.plan's native launch list: SDMI_SAMPLE_ISSUE=plan) and replayed
per step with no host work.

Everything a step needs lives on the device: the model's timestep is an int64 device scalar read by the
time-embedding kernel; the DDPM step kernel (sdmi_ddpm_prev) decrements it after the step, the DDIM step kernel
(sdmi_ddim_prev_dev) reads its (t, t_prev) pair from device tables through a device step index and moves both down;
the noise comes from the Philox kernel (sdmi_randn) keyed by (seed, device draw counter) that advances per replay;
x_t is updated in place. The reference instead builds t on the host, draws the noise with the host generator (DDPM:
on the CPU, scheduler :72) and syncs on `t == 0` every step.

A model that does not run on the fused engine (a swapped leaf, SURVEY.md §8(b), or sdmi_leaf_path = True) is
sampled stepwise through its own forward (`model(x, t, cond)`), with the same step kernels and noise."""
import ctypes
import os

import numpy as np
import torch

from . import _lib
from . import kernels as K
from .module_glue import engine_path_ok
from .plan import StepPlan


class _Loop:
    """Shared state of a captured loop: the model binding (fused engine, or a stepwise model call), x_t / noise /
    device-counter buffers and the recorded plan."""

    def __init__(self, model, shape, cond_input, seed):
        dev = next(model.parameters()).device
        if dev.type != "cuda":
            raise RuntimeError("the sampling loop runs on the MI355X HIP path only (move the model to cuda)")
        self.dev = dev
        self.model = model
        # the fused engine only when the model's forward would use it (no swapped / foreign leaves, no leaf override)
        self.fused = hasattr(model, "_sdmi") and engine_path_ok(model)
        self.eng = model._sdmi.ensure(dev) if self.fused else None
        B, C, H, W = shape
        self.shape = (B, C, H, W)
        self.xt = torch.empty(shape, dtype=torch.float32, device=dev)
        self.z = torch.empty_like(self.xt)
        self.eps = None  # the model output of the last step (a buffer of the recorded plan)
        self.t = torch.zeros(1, dtype=torch.int64, device=dev)
        self.offset = torch.zeros(1, dtype=torch.int64, device=dev)  # Philox draw counter (uint64 bits)
        self.seed = int(seed)
        c = cond_input or {}
        self.cond = cond_input
        self.text, self.mask, self.klass = c.get("text"), c.get("image"), c.get("class")
        self.plan = None
        # captured issue: "graph" (default) -- the reverse step as ONE hipGraph launch (torch.cuda.CUDAGraph of the
        # eager step; one stream, since inference keeps the context branch inline); "plan" -- sdmi.plan's
        # native launch list re-issued per step. Both bit-identical to the stepwise loop; the graph removes the
        # per-launch host issue that bounds the small-batch step (scripts/sample_graph_probe.py)
        self.issue = os.environ.get("SDMI_SAMPLE_ISSUE", "graph")
        if self.issue not in ("graph", "plan"):
            raise ValueError(f"SDMI_SAMPLE_ISSUE={self.issue!r}: graph or plan")
        self.graph = None
        self.ctx_cache = None

    def _refresh(self):
        """Pack the current weights (plain kernel launches into the engine's fixed buffers, outside the plan): a loop
        reused after a training update or an EMA swap samples with the weights of the moment it runs. Parameters
        REPLACED rather than updated in place (load_state_dict(assign=True), .to(), ...) rebind the engine; a new
        engine or a re-allocated pack buffer drops the recorded graph / plan, which hold the old pointers."""
        if self.fused:
            eng = self.model._sdmi.ensure(self.dev)
            buf = getattr(getattr(eng, "pack", None), "buf", None)
            if eng is not self.eng:
                self.eng = eng
                self._drop_recording()
            self.eng.refresh_weights()
            nbuf = getattr(getattr(self.eng, "pack", None), "buf", None)
            if nbuf is not buf:  # refresh_weights re-finalised the pack into a new buffer
                self._drop_recording()
            # the context branch (text -> context_proj -> every cross-attention's k|v) is the same for every step of
            # the loop: computed once per run into fixed buffers (UNetEngine.context_cache) instead of per step
            if self.text is not None and hasattr(self.eng, "context_cache"):
                self.ctx_cache = self.eng.context_cache(self.text, self.ctx_cache)

    def _drop_recording(self):
        self.graph = None
        self.plan = None
        self.ctx_cache = None

    def _model_eps(self):
        B, C, H, W = self.shape
        if self.fused:
            kw = {"ctx_cache": self.ctx_cache} if self.ctx_cache is not None else {}
            pred, _ = self.eng.forward(self.xt, self.t, self.text, self.mask, need_backward=False, klass=self.klass,
                                       **kw)
            self.eps = self.eng.pred_to_nchw(pred, B, H, W)
        else:
            with torch.no_grad():
                tt = self.t.expand(B)
                out = self.model(self.xt, tt) if self.cond is None else self.model(self.xt, tt, self.cond)
            self.eps = out.float().contiguous()

    @staticmethod
    def fresh_draw():
        """A random 62-bit starting draw counter from torch's default generator: torch.manual_seed governs it, and runs
        started from different counters draw disjoint Philox streams (a run uses `steps` consecutive counters)."""
        return int(torch.randint(0, 1 << 62, (1,)).item())

    def _draw(self):
        _lib.check(_lib.lib().sdmi_randn(self.z.data_ptr(), self.xt.numel(), ctypes.c_ulonglong(self.seed),
                                         self.offset.data_ptr(), 1, K._stream()), "sdmi_randn")

    def _iterate(self, steps, captured):
        # the stepwise (foreign-leaf) path reads device scalars through torch ops: never recorded
        captured = captured and self.fused
        for _ in range(steps):
            if not captured:
                self._step()
            elif self.issue == "graph":
                if self.graph is None:  # the first step runs eagerly, then the step is captured (capture runs nothing)
                    self._step()
                    self.graph = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(self.graph):
                        self._step()
                else:
                    self.graph.replay()
            elif self.plan is None:  # the first step is recorded while it runs
                self.plan = StepPlan(self._step, self.dev)
            else:
                self.plan.replay()


class DDPMSampleLoop(_Loop):
    def __init__(self, model, scheduler, shape, cond_input=None, seed=0):
        """model: a drop-in denoiser module (models.unet_cond_base.Unet / unet_base.Unet / transformer.DIT) already
        on the GPU; scheduler: scheduler.linear_noise_scheduler.LinearNoiseScheduler; shape: (B, C, H, W) latents;
        cond_input: the model's condition dict (text / image / class), fixed for the whole loop."""
        super().__init__(model, shape, cond_input, seed)
        self.T = scheduler.num_timesteps
        self.tab = scheduler.tables(self.dev)
        self.x0 = torch.empty_like(self.xt)

    def _step(self):
        self._model_eps()
        self._draw()
        tab = self.tab
        _lib.check(_lib.lib().sdmi_ddpm_prev(self.xt.data_ptr(), self.eps.data_ptr(), self.z.data_ptr(),
                                             self.xt.numel(), self.t.data_ptr(), tab["betas"].data_ptr(),
                                             tab["alphas"].data_ptr(), tab["alpha_cum_prod"].data_ptr(),
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
        self._refresh()
        self.reset(x_T, t_start)
        self._iterate(self.T if steps is None else int(steps), captured)
        return self.xt, self.x0


def ddim_time_steps(T, steps, method="linear"):
    """DDIMSampler.forward's timestep pairs (scheduler/linear_noise_scheduler.py:231-242): "linear" range(0, T, T //
    steps) or "quadratic" int32(linspace(0, sqrt(0.8 T), steps)^2), both + 1; previous = [0] + ts[:-1]."""
    if method == "linear":
        ts = np.asarray(list(range(0, T, T // steps)))
    elif method == "quadratic":
        ts = (np.linspace(0, np.sqrt(T * 0.8), steps) ** 2).astype(np.int32)
    else:
        raise NotImplementedError(f"sampling method {method} is not implemented!")
    ts = ts + 1
    return ts, np.concatenate([[0], ts[:-1]])


class DDIMSampleLoop(_Loop):
    """DDIMSampler.forward (reference :209-256) with the model, the DDIM update and the per-step noise
    (torch.randn_like at :200, here device Philox) recorded once and replayed `steps` times."""

    def __init__(self, model, alpha_t_bar, shape, cond_input=None, steps=50, method="linear", eta=0.0, seed=0):
        """alpha_t_bar: the sampler's fp32 cumulative-product table (DDIMSampler.alpha_t_bar, from linspace(beta))."""
        super().__init__(model, shape, cond_input, seed)
        self.steps = int(steps)
        self.eta = float(eta)
        ts, tp = ddim_time_steps(len(alpha_t_bar), self.steps, method)
        # the reference's loop reads pairs i = steps - 1 .. 0 only (linear spacing can yield more when T % steps != 0)
        if len(ts) < self.steps:
            raise ValueError(f"{method} time steps: {len(ts)} pairs for steps={self.steps}")
        ts, tp = ts[:self.steps], tp[:self.steps]
        if int(ts.max()) >= len(alpha_t_bar):  # the reference would raise an IndexError in its gather
            raise IndexError(f"DDIM timestep {int(ts.max())} out of range for T={len(alpha_t_bar)}")
        self.ts = torch.as_tensor(ts, dtype=torch.int64).to(self.dev)
        self.tp = torch.as_tensor(tp, dtype=torch.int64).to(self.dev)
        self.abar = alpha_t_bar.to(device=self.dev, dtype=torch.float32).contiguous()
        self.idx = torch.zeros(1, dtype=torch.int64, device=self.dev)

    def _step(self):
        self._model_eps()
        self._draw()
        # elementwise and in place: x_{t-1} overwrites x_t (the next step's model input)
        _lib.check(_lib.lib().sdmi_ddim_prev_dev(self.xt.data_ptr(), self.eps.data_ptr(), self.z.data_ptr(),
                                                 self.xt.numel(), self.ts.data_ptr(), self.tp.data_ptr(),
                                                 self.idx.data_ptr(), self.t.data_ptr(), self.abar.data_ptr(),
                                                 self.eta, self.xt.data_ptr(), 1, K._stream()), "sdmi_ddim_prev_dev")

    def reset(self, x_T, draw=0):
        self.xt.copy_(x_T)
        self.idx.fill_(self.steps - 1)
        self.t.copy_(self.ts[self.steps - 1:self.steps])
        self.offset.fill_(int(draw))

    def run(self, x_T, captured=True, draw=0):
        """The whole reversed loop (i = steps - 1 .. 0) from x_T; returns x_0 (the loop's buffer). `draw` is the Philox
        draw counter the run starts at: runs from the same (seed, draw) repeat their noise exactly; fresh_draw() gives
        a run noise of its own."""
        self._refresh()
        self.reset(x_T, draw)
        self._iterate(self.steps, captured)
        return self.xt
