"""Glue between the nn.Module surface (models/) and the HIP engines: flat parameter adoption and the
autograd Function whose forward/backward run a denoiser engine (UNetEngine or DiTEngine)."""
import torch

from . import _lib
from .store import FlatStore
from .unet_engine import UNetEngine
from .dit_engine import DiTEngine, dit_flat_order


def _require_gpu(t):
    if not t.is_cuda:
        raise RuntimeError("the sdmi denoisers run on the MI355X HIP path only (move the model and inputs to cuda)")
    _lib.lib()  # fail loudly when the extension is missing


class EngineHolder:
    """Per-module state: flat store the nn.Parameters live in, and the engine bound to it.
    base: "cond" / "uncond" (UNet) or "dit"."""

    def __init__(self, module, cfg, base):
        self.module = module
        self.cfg = cfg
        self.base = base
        self.store = None
        self.engine = None
        self._packed_sig = None

    def ensure(self, device):
        params = dict(self.module.named_parameters())
        adopted = self.store is not None and all(
            params[k].data_ptr() == self.store.p[k].data_ptr() for k in self.store.order)
        if not adopted:
            shapes = {k: tuple(v.shape) for k, v in params.items()}
            order = dit_flat_order(self.cfg, list(shapes)) if self.base == "dit" else None
            store = FlatStore(shapes, self.cfg, device, with_grads=False, order=order)
            with torch.no_grad():
                for k in store.order:
                    store.p[k].copy_(params[k].detach())
            for k in store.order:  # the Parameter objects keep their identity (optimizers stay valid)
                params[k].data = store.p[k]
            self.store = store
            if self.base == "dit":
                self.engine = DiTEngine(self.cfg, store.p, None, im_channels=self.module.im_channels)
            else:
                self.engine = UNetEngine(self.cfg, store.p, None, base=self.base, im_channels=self.module.im_channels)
            self._packed_sig = None
        return self.engine

    def refresh(self, params):
        """Repack the bf16 GEMM-layout weights (the cast autocast performs on every forward).
        Grad-enabled calls (training) repack unconditionally: updates written through `.data` -- the reference's EMA
        `.data.mul_().add_()` (train_ddpm_cond_celebhq_multi_gpu.py:376-378), PercentOptimizerFP / DDFP SGD
        (cim_layers/IBA_optimizer.py:67) -- do not bump a tensor's version counter, and one batched pack launch is
        cheap next to a training step. Under torch.no_grad (sampling loops, tools/sample_ddpm_*.py: 1000 forwards and
        no updates) the pack is skipped while no parameter's version changed; call invalidate() after writing
        weights through `.data` between no-grad forwards."""
        sig = tuple(p._version for p in params)
        if torch.is_grad_enabled() or sig != self._packed_sig:
            self.engine.refresh_weights()
            self._packed_sig = sig

    def invalidate(self):
        """Force a repack at the next forward (weights changed behind the version counter, e.g. via `.data`)."""
        self._packed_sig = None


def invalidate_module(module):
    """Weights of `module` were written behind the version counter (`.data`): repack everything at the next forward
    (the fused engine's packs, the leaf path's per-module packs, the VQVAE training engine's)."""
    from . import leaf
    for m in module.modules():
        h = getattr(m, "_sdmi", None)
        if isinstance(h, EngineHolder):
            h.invalidate()
        if hasattr(m, "_tsig"):
            m._tsig = None
    leaf.invalidate_packs(module)


def engine_path_ok(model):
    """True when `model` (a drop-in denoiser) runs on the fused whole-network engine: no sdmi_leaf_path override and
    every leaf an exact engine type (sdmi.leaf.engine_ok with the model's own container classes)."""
    if getattr(model, "sdmi_leaf_path", False):
        return False
    check = getattr(model, "_sdmi_engine_ok", None)
    return bool(check()) if check is not None else False


class DenoiserFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, holder, x, t, text, mask, klass, *params):
        eng = holder.engine
        B, C, H, W = x.shape
        pred, tape = eng.forward(x, t, text, mask, need_backward=True, klass=klass)
        out = eng.pred_to_nchw(pred, B, H, W)
        ctx.holder = holder
        ctx.tape = tape
        return out

    @staticmethod
    def backward(ctx, dout):
        holder = ctx.holder
        eng = holder.engine
        store = holder.store
        dpred = eng.dpred_from_nchw(dout.float().contiguous())
        gflat = torch.empty(store.numel, dtype=torch.float32, device=dout.device)
        gviews = {k: store.view(gflat, k) for k in store.order}
        eng.backward(ctx.tape, dpred, grads=gviews)
        ctx.tape = None
        names = [k for k, _ in holder.module.named_parameters()]
        return (None, None, None, None, None, None) + tuple(gviews[k] for k in names)


UNetFunction = DenoiserFunction


def run_unet(module, holder, x, t, text=None, mask=None, klass=None):
    _require_gpu(x)
    eng = holder.ensure(x.device)
    params = [p for _, p in module.named_parameters()]
    holder.refresh(params)
    if torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in params)):
        return DenoiserFunction.apply(holder, x, t, text, mask, klass, *params)
    # inference (torch.no_grad sampling loops): no backward tape, no saved activations
    B, C, H, W = x.shape
    pred, _ = eng.forward(x, t, text, mask, need_backward=False, klass=klass)
    return eng.pred_to_nchw(pred, B, H, W)


run_denoiser = run_unet
