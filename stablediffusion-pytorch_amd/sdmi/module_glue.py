"""Glue between the nn.Module surface (models/) and the HIP engine: flat parameter adoption and the
autograd Function whose forward/backward run UNetEngine."""
import torch

from . import _lib
from . import kernels as K
from .store import FlatStore
from .unet_engine import UNetEngine


def _require_gpu(t):
    if not t.is_cuda:
        raise RuntimeError("the sdmi UNet runs on the MI355X HIP path only (move the model and inputs to cuda)")
    _lib.lib()  # fail loudly when the extension is missing


class EngineHolder:
    """Per-module state: flat store the nn.Parameters live in, and the engine bound to it."""

    def __init__(self, module, cfg, base):
        self.module = module
        self.cfg = cfg
        self.base = base
        self.store = None
        self.engine = None

    def ensure(self, device):
        params = dict(self.module.named_parameters())
        adopted = self.store is not None and all(
            params[k].data_ptr() == self.store.p[k].data_ptr() for k in self.store.order)
        if not adopted:
            shapes = {k: tuple(v.shape) for k, v in params.items()}
            store = FlatStore(shapes, self.cfg, device, with_grads=False)
            with torch.no_grad():
                for k in store.order:
                    store.p[k].copy_(params[k].detach())
            for k in store.order:  # the Parameter objects keep their identity (optimizers stay valid)
                params[k].data = store.p[k]
            self.store = store
            self.engine = UNetEngine(self.cfg, store.p, None, base=self.base,
                                     im_channels=self.module.im_channels)
        return self.engine


class UNetFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, holder, x, t, text, mask, *params):
        eng = holder.engine
        eng.refresh_weights()
        B, C, H, W = x.shape
        pred, tape = eng.forward(x, t, text, mask, need_backward=torch.is_grad_enabled() or True)
        out = torch.empty(B, C, H, W, dtype=torch.float32, device=x.device)
        _lib.check(_lib.lib().sdmi_nhwc_to_nchw(pred.data_ptr(), 1, 8, B, C, H * W, out.data_ptr(), K._stream()),
                   "sdmi_nhwc_to_nchw")
        ctx.holder = holder
        ctx.tape = tape
        ctx.shape = (B, C, H, W)
        return out

    @staticmethod
    def backward(ctx, dout):
        holder = ctx.holder
        eng = holder.engine
        store = holder.store
        B, C, H, W = ctx.shape
        d = dout.float().contiguous()
        dpred = torch.empty(B * H * W, 8, dtype=torch.bfloat16, device=d.device)
        _lib.check(_lib.lib().sdmi_nchw_to_nhwc_bf16(d.data_ptr(), B, C, H * W, dpred.data_ptr(), 8, K._stream()),
                   "sdmi_nchw_to_nhwc_bf16")
        gflat = torch.empty(store.numel, dtype=torch.float32, device=d.device)
        gviews = {k: store.view(gflat, k) for k in store.order}
        eng.backward(ctx.tape, dpred, grads=gviews)
        ctx.tape = None
        names = [k for k, _ in holder.module.named_parameters()]
        return (None, None, None, None, None) + tuple(gviews[k] for k in names)


def run_unet(module, holder, x, t, text=None, mask=None):
    _require_gpu(x)
    holder.ensure(x.device)
    params = [p for _, p in module.named_parameters()]
    return UNetFunction.apply(holder, x, t, text, mask, *params)
