"""Glue between the nn.Module surface (models/) and the HIP engines: flat parameter adoption and the
autograd Functions whose forward/backward run a denoiser engine (UNetEngine or DiTEngine).

Two backward forms (same kernels, same gradients):
* DenoiserFunction: one autograd node; every parameter gradient is handed to autograd when the whole engine backward
  has been issued.
* StagedBackward (data-parallel callers): the engine backward split into a chain of autograd nodes, each handing out
  the gradients that became final in the previous segment. The reference wraps the model in
  DistributedDataParallel (train_ddpm_cond_celebhq_multi_gpu.py:257-263) and relies on its per-parameter autograd
  hooks to start bucket all-reduces during the backward (:362); with a single node every hook fires at the end and
  nothing overlaps. Used when torch.distributed is initialised with world size > 1 (module attribute
  `sdmi_staged_backward` = True / False overrides)."""
import torch
import torch.distributed as dist

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
        self._gflat = None
        self._stages = {}  # tape-label signature -> segment plan of the staged backward

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

    def grad_buffer(self, device):
        """The flat fp32 buffer a backward writes every parameter gradient into (store order), reused across
        backwards (verdict r5: a fresh 474 MB buffer per backward at the full cond-UNet). autograd hands the per-
        parameter views to `.grad` without a copy when `.grad` is None (zero_grad(set_to_none=True), the reference's
        loops), so a `.grad` that still aliases the buffer -- gradient accumulation without zeroing, where the next
        backward is ADDED into `.grad` -- gets a fresh buffer instead of being overwritten."""
        g = self._gflat
        if g is not None and g.device == torch.device(device):
            sp = g.untyped_storage().data_ptr()
            if not any(p.grad is not None and p.grad.device == g.device and p.grad.untyped_storage().data_ptr() == sp
                       for p in self.module.parameters()):
                return g
        self._gflat = torch.empty(self.store.numel, dtype=torch.float32, device=device)
        return self._gflat


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
        gflat = holder.grad_buffer(dout.device)
        gviews = {k: store.view(gflat, k) for k in store.order}
        eng.backward(ctx.tape, dpred, grads=gviews)
        ctx.tape = None
        names = [k for k, _ in holder.module.named_parameters()]
        return (None, None, None, None, None, None) + tuple(gviews[k] for k in names)


UNetFunction = DenoiserFunction


def _final_sets(holder, tape):
    """Segment plan of a staged backward: [(stop token, keys final by then)] in backward order, plus the keys final
    only when the engine backward is exhausted. Tokens are what the engine's backward_steps() yields (UNet: tape
    position; DiT: layer index). Consecutive finalisations are merged into segments of >= 1/8 of the parameter bytes,
    so a step pays at most ~8 segment boundaries."""
    from .store import param_label
    names = [k for k, _ in holder.module.named_parameters()]
    store = holder.store
    if holder.base == "dit":
        n_layers = holder.engine.L["n_layers"]

        def layer_of(k):
            if k.startswith("proj_out"):
                return n_layers  # final with the first yielded layer
            if k.startswith("transformer_layers.") and ".adaptive_norm_layer." not in k:
                return int(k.split(".")[1])
            return None  # adaLN tables, t_proj, patch embedding, conditioning: the tail
        tokens = list(range(n_layers - 1, -1, -1))
        at = {}
        for k in names:
            li = layer_of(k)
            if li is not None:
                at.setdefault(min(li, n_layers - 1), []).append(k)
    else:
        done_at = {}
        for k in range(len(tape) - 1, -1, -1):  # a label is complete at its earliest tape entry
            done_at[tape[k][1]["label"]] = k
        tokens = list(range(len(tape) - 1, -1, -1))
        at = {}
        for key in names:
            k = done_at.get(param_label(key))
            if k is not None and k > 0:  # (label finished at entry 0: with the tail)
                at.setdefault(k, []).append(key)
    total = sum(store.offsets[k][1] for k in names)
    seg, segs, acc = [], [], 0
    for tok in tokens:
        for key in at.get(tok, []):
            seg.append(key)
            acc += store.offsets[key][1]
        if seg and acc * 8 >= total:
            segs.append((tok, seg))
            seg, acc = [], 0
    given = {k for _, ks in segs for k in ks}
    tail = [k for k in names if k not in given]
    return segs, tail


class _StagedRun:
    """One staged backward: the engine's backward generator driven by the chain of _Stage nodes."""

    def __init__(self, holder, tape_ctx, shape, segs, tail):
        self.holder, self.ctx, self.shape = holder, tape_ctx, shape
        self.segs, self.tail = segs, tail
        self.gen = None
        self.tok = None
        self.events = []
        self.handed = 0  # segments whose gradients have been returned to autograd (test / overlap evidence)

    def begin(self, dout):
        h = self.holder
        eng, store = h.engine, h.store
        dpred = eng.dpred_from_nchw(dout.float().contiguous())
        gflat = h.grad_buffer(dout.device)
        self.gviews = {k: store.view(gflat, k) for k in store.order}
        self.gen = eng.backward_steps(self.ctx, dpred, grads=self.gviews)

    def _advance(self, stop):
        """Run the engine backward until it has yielded a token <= stop (tokens decrease; the DiT engine yields only
        where a group of layers' weight gradients has been issued, so a stop may be passed rather than hit)."""
        if self.tok is not None and self.tok <= stop:
            return
        for tok in self.gen:
            self.tok = tok
            if tok <= stop:
                return
        raise RuntimeError(f"staged backward: the engine backward ended before token {stop}")

    def _sides(self):
        return getattr(self.holder.engine, "sides", None) or []

    def segment(self, j):
        """Run the engine backward to stop j and return the gradients that were final at stop j - 1 (their side-
        stream work was issued a whole segment ago: waiting for it on the current stream rarely stalls)."""
        from . import plan
        cur = torch.cuda.current_stream()
        self._advance(self.segs[j][0])
        evs = []
        for sd in self._sides():
            ev = torch.cuda.Event()
            plan.record_event(ev, sd)
            evs.append(ev)
        self.events.append(evs)
        if j == 0:
            return ()
        for ev in self.events[j - 1]:
            plan.wait_event(cur, ev)
        self.handed += 1
        return tuple(self.gviews[k] for k in self.segs[j - 1][1])

    def last(self):
        """Exhaust the engine backward (its own join of every side stream) and return the rest."""
        for _ in self.gen:
            pass
        keys = (self.segs[-1][1] if self.segs else []) + self.tail
        self.handed += 1
        self.gen = None
        return tuple(self.gviews[k] for k in keys)


class _StageOut(torch.autograd.Function):
    """Last node of the forward chain (its backward runs first): produces the prediction; backward starts the engine
    backward and runs segment 0."""

    @staticmethod
    def forward(ctx, run, h, *params):
        ctx.run = run
        eng = run.holder.engine
        B, H, W, pred = run.shape
        return eng.pred_to_nchw(pred, B, H, W)

    @staticmethod
    def backward(ctx, dout):
        run = ctx.run
        run.begin(dout)
        if run.segs:
            run.segment(0)  # (segment 0 hands out nothing: its gradients go out with segment 1)
        return None, torch.zeros(0, device=dout.device)


class _Stage(torch.autograd.Function):
    """Middle node j: runs segment j, hands out segment j - 1's gradients."""

    @staticmethod
    def forward(ctx, run, j, h, *params):
        ctx.run, ctx.j = run, j
        return h.new_zeros(0)

    @staticmethod
    def backward(ctx, dh):
        return (None, None, torch.zeros(0, device=dh.device)) + ctx.run.segment(ctx.j)


class _StageFirst(torch.autograd.Function):
    """First node of the forward chain (its backward runs last): finishes the engine backward."""

    @staticmethod
    def forward(ctx, run, *params):
        ctx.run = run
        return params[0].new_zeros(0) if params else torch.zeros(0, device="cuda")

    @staticmethod
    def backward(ctx, dh):
        return (None,) + ctx.run.last()


def staged_apply(holder, pred, tape_ctx, B, H, W):
    """The prediction as the output of a chain of autograd nodes over the parameters (see the module docstring).
    Node order in the backward: _StageOut (segment 0), _Stage j = 1 .. n-1, _StageFirst (the rest)."""
    tape = tape_ctx.get("tape") if isinstance(tape_ctx, dict) else None
    sig = tuple(c.get("label") for _, c in tape) if tape is not None else ("dit",)
    if sig not in holder._stages:
        holder._stages[sig] = _final_sets(holder, tape)
    segs, tail = holder._stages[sig]
    named = dict(holder.module.named_parameters())
    run = _StagedRun(holder, tape_ctx, (B, H, W, pred), segs, tail)
    # forward chain: first node owns the gradients handed out last
    keys_last = (segs[-1][1] if segs else []) + tail
    h = _StageFirst.apply(run, *[named[k] for k in keys_last])
    for j in range(len(segs) - 1, 0, -1):
        h = _Stage.apply(run, j, h, *[named[k] for k in segs[j - 1][1]])
    out = _StageOut.apply(run, h)
    holder.last_run = run
    return out


def staged_enabled(module):
    flag = getattr(module, "sdmi_staged_backward", None)
    if flag is not None:
        return bool(flag)
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def run_unet(module, holder, x, t, text=None, mask=None, klass=None):
    _require_gpu(x)
    eng = holder.ensure(x.device)
    params = [p for _, p in module.named_parameters()]
    holder.refresh(params)
    if torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in params)):
        if staged_enabled(module):
            B, C, H, W = x.shape
            pred, tape_ctx = eng.forward(x, t, text, mask, need_backward=True, klass=klass)
            return staged_apply(holder, pred, tape_ctx, B, H, W)
        return DenoiserFunction.apply(holder, x, t, text, mask, klass, *params)
    # inference (torch.no_grad sampling loops): no backward tape, no saved activations
    B, C, H, W = x.shape
    pred, _ = eng.forward(x, t, text, mask, need_backward=False, klass=klass)
    return eng.pred_to_nchw(pred, B, H, W)


run_denoiser = run_unet
