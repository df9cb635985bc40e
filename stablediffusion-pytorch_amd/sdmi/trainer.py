"""The reference's DDPM training step (train_ddpm_cond_celebhq_multi_gpu.py:299-378) as one stream of
gfx950 kernels:

    add_noise -> UNet forward -> MSE (x loss scale) -> UNet backward
      (-> bucketed RCCL all-reduce overlapped with the backward, N > 1)
    -> unscale / clip_grad_norm(1.0) / non-finite skip -> Adam(lr) -> EMA(0.9999)
    -> bf16 GEMM-layout weight repack for the next step

Master weights, Adam moments and the EMA copy are flat fp32 buffers (sdmi.store.FlatStore order), the
GradScaler state (scale, growth tracker, step, skip flag) lives on the device, so a step never
synchronises with the host (the reference's .item()/isfinite syncs at :348-371 become device flags)."""
import math
import os

import torch
import torch.distributed as dist

from . import _lib
from . import kernels as K
from . import plan
from . import streams
from .reducer import BucketReducer, NormBlocks
from .store import FlatStore, param_label, unet_gemm_natural
from .unet_engine import UNetEngine
from .dit_engine import DiTEngine, dit_flat_order

# state vector layout (see csrc/optim.hip)
S_NORM, S_COEF, S_SCALE, S_GROWTH, S_STEP, S_SKIP, S_LOSS, S_DPFLAG = range(8)


def scheduler_tables(num_timesteps, beta_start, beta_end):
    """Reference scheduler tables (scheduler/linear_noise_scheduler.py:18-24), built on the host in fp32."""
    betas = torch.linspace(beta_start ** 0.5, beta_end ** 0.5, num_timesteps) ** 2
    abar = torch.cumprod(1. - betas, dim=0)
    return torch.sqrt(abar), torch.sqrt(1 - abar)


class NormParts:
    """clip_grad_norm_'s sum of squares in pieces overlapped with the backward (one GPU): as soon as the backward has
    finalised a >= `chunk` slice of the flat gradient buffer (the same watermarks the data-parallel reducer uses), its
    block partials (NormBlocks: fixed blocks at absolute flat offsets, the watermark rounded down to a block boundary)
    run on a stream of their own behind every gradient producer; the last slice and the finalisation run on the compute
    stream, so the step boundary (backward end -> norm -> first optimizer chunk -> next forward) no longer waits for a
    full pass over the 474 MB of gradients. Every block's partial depends only on its data and the finalisation sums
    them in block order: bitwise the norm of one whole-buffer pass (sdmi_clip_unscale) and of the data-parallel
    reducer's per-bucket pieces."""

    def __init__(self, grads, numel, producers=(), chunk_elems=16 << 20, stream=None):
        self.g, self.numel = grads, numel
        self.chunk = chunk_elems
        self.producers = list(producers)
        self.stream = stream or streams.new_stream(grads.device)
        self.blocks = NormBlocks(numel, grads.device)
        self.reset()

    def reset(self):
        self.launched = 0

    def ready(self, upto):
        """Gradients at flat offsets < upto are final (called during the backward)."""
        upto = self.blocks.floor(min(upto, self.numel))
        if upto - self.launched < self.chunk:
            return
        for st in [torch.cuda.current_stream(self.g.device)] + self.producers:
            ev = torch.cuda.Event()
            plan.record_event(ev, st)
            plan.wait_event(self.stream, ev)
        self.blocks.launch(self.g, self.launched, upto, self.stream)
        self.launched = upto

    def finish(self, max_norm, state, growth, skip_mode, grad_div):
        """After the backward (side streams joined into the current stream): the rest, then clip / skip / scaler."""
        cur = torch.cuda.current_stream(self.g.device)
        if self.launched < self.numel:
            self.blocks.launch(self.g, self.launched, self.numel, cur)
        plan.wait_stream(cur, self.stream)
        finalize_norm(self.blocks, max_norm, state, growth, skip_mode, grad_div)


def finalize_norm(blocks, max_norm, state, growth, skip_mode, grad_div):
    """clip / skip / GradScaler update from a complete NormBlocks partial array (current stream)."""
    _lib.check(_lib.lib().sdmi_clip_finalize(blocks.partials.data_ptr(), blocks.n, max_norm, state.data_ptr(), growth,
                                             skip_mode, grad_div, K._stream()), "sdmi_clip_finalize")


class DDPMTrainer:
    """base: "cond" / "uncond" (UNet, train_ddpm_cond_celebhq_multi_gpu.py:299-378, EMA 0.9999) or "dit"
    (Model_DiT_12L_train.py:300-375: same step, no EMA -- pass ema_decay=None -- and lr 1e-4)."""

    def __init__(self, cfg, state_dict, device, *, base="cond", lr=1e-5, betas=(0.9, 0.999), eps=1e-8,
                 max_grad_norm=1.0, ema_decay=0.9999, init_scale=65536.0, growth_interval=2000,
                 sched=(1000, 0.00085, 0.012), group=None, bucket_bytes=64 << 20, force_reducer=False,
                 grad_wire=None, single_stream=False):
        """single_stream: every kernel on the current stream (no weight-gradient / context / optimizer side streams:
        single-stream hipGraph capture, isolated GEMM timing)."""
        self.cfg = cfg
        self.base = base
        self.device = torch.device(device)
        shapes = {k: tuple(v.shape) for k, v in state_dict.items()}
        order = dit_flat_order(cfg, list(shapes)) if base == "dit" else None
        self.group = group
        self.world = dist.get_world_size(group) if (group is not None or dist.is_initialized()) else 1
        # N > 1: one fp32 slot after the gradients carries this rank's non-finite-loss flag through the all-reduce
        # UNet: 3x3 / down-sampling conv weights in GEMM-natural (co, kh, kw, ci) order (store.unet_gemm_natural)
        nat = unet_gemm_natural if base != "dit" else None
        self.store = FlatStore(shapes, cfg, self.device, order=order, grad_tail=4 if self.world > 1 else 0, natural=nat)
        self.store.load(state_dict)
        if self.world > 1:
            # DistributedDataParallel broadcasts rank 0's parameters when it wraps the model
            # (train_ddpm_cond_celebhq_multi_gpu.py:257-263): every replica (and its EMA copy) starts from them
            src = 0 if group is None or group is dist.group.WORLD else dist.get_global_rank(group, 0)
            dist.broadcast(self.store.params, src=src, group=group)
        # EMA copy (train_ddpm_cond_celebhq_multi_gpu.py:376-378); none for the DiT trainer (commented out at
        # Model_DiT_12L_train.py:377-379): the fused optimizer then skips the EMA stream entirely
        self.ema = self.store.params.clone() if ema_decay is not None else None
        self.m = torch.zeros_like(self.store.params)
        self.v = torch.zeros_like(self.store.params)
        self.state = torch.tensor([0, 0, init_scale, 0, 0, 0, 0, 0], dtype=torch.float32, device=self.device)
        self.hp = dict(lr=lr, b1=betas[0], b2=betas[1], eps=eps, clip=max_grad_norm, ema=ema_decay,
                       growth=growth_interval)
        if base == "dit":
            self.engine = DiTEngine(cfg, self.store.p, self.store.g, single_stream=single_stream)
        else:
            # latent channels from the state dict (4 for CelebHQ, the VQVAE's z_channels in general: 3 for MNIST)
            self.engine = UNetEngine(cfg, self.store.p, self.store.g, base=base,
                                     im_channels=shapes["conv_out.weight"][0], single_stream=single_stream)
        self.num_timesteps = sched[0]
        sa, s1a = scheduler_tables(*sched)
        self.sqrt_abar, self.sqrt_1m_abar = sa.to(self.device), s1a.to(self.device)
        # force_reducer: run the bucketed all-reduce even at world size 1 (exercises RCCL + plan replay on one GPU)
        # gradient wire format of the all-reduce: fp32 (the reference's DDP) unless grad_wire / SDMI_GRAD_WIRE = bf16
        self.grad_wire = grad_wire or os.environ.get("SDMI_GRAD_WIRE", "fp32")
        # the reducer also produces the gradient norm: each bucket's block partials right after its all-reduce
        self.red_norm = (NormBlocks(self.store.numel, self.device)
                         if (self.world > 1 or force_reducer) and self.device.type == "cuda" else None)
        # the reducer (and below the one-GPU norm pieces) run on the engine's context stream, idle in the backward,
        # where there is one: a process gets four hardware queues (sdmi/streams.py) and the step's main, two weight-
        # gradient and context streams already hold them (forced-reducer step 14.99 -> 14.75 ms with this alone;
        # SDMI_RED_STREAM / SDMI_NORM_STREAM = own: a stream of their own)
        red_stream = (getattr(self.engine, "ctx_stream", None)
                      if os.environ.get("SDMI_RED_STREAM", "ctx") == "ctx" else None)
        self.reducer = (BucketReducer(self.store.grads, group, bucket_bytes, wire=self.grad_wire, norm=self.red_norm,
                                      stream=red_stream)
                        if self.world > 1 or force_reducer else None)
        self.tail_events = None  # (after backward, after the all-reduce drain): set by measure_exchange_tail()
        # one GPU: the gradient norm in pieces overlapped with the backward.
        # With N > 1 the norm needs the all-reduced gradients: the reducer computes it bucket by bucket.
        self.norm_parts = None
        if self.world == 1 and self.reducer is None and self.device.type == "cuda":
            self.norm_parts = NormParts(self.store.grads, self.store.numel,
                                        getattr(self.engine, "sides", None) or [],
                                        stream=(getattr(self.engine, "ctx_stream", None)
                                                if os.environ.get("SDMI_NORM_STREAM", "ctx") == "ctx" else None))
        if self.reducer is not None and getattr(self.engine, "side", None) is not None:
            self.reducer.producers.extend(getattr(self.engine, "sides", None) or [self.engine.side])
        self._progress = None
        # Optimizer + weight packing pipelined against the next step's forward: the flat buffer is cut into
        # forward-ordered chunks; after the (global) clip, Adam + EMA + packing run chunk by chunk on the engine's
        # side stream, each chunk ending in an event that the engine waits for only where the forward first reads
        # one of that chunk's parameters or packed weights (UNet engine, 6 chunks).
        # DiT: the forward's first GEMM (every layer's adaLN table) needs the largest chunk at once, so pipelining
        # measured no gain there (4.00 ms/step unchunked vs 4.04-4.07 at 6 chunks; round 4: 3.53 / 3.53 unchunked vs
        # 3.55 / 3.55, 3.53 / 3.53, 3.54 / 3.53 at 2 / 3 / 6 forward-ordered chunks): one chunk
        nchunks = 1 if base == "dit" else 6
        self.opt_ranges = None
        if nchunks > 1 and getattr(self.engine, "side", None) is not None:
            # lead chunks (the runs the next forward reads first, then its first two blocks): same-box A/B
            # 13.88 / 13.82 -> 13.85 / 13.81 ms, the step-start wait for the first chunk 101 -> 30 us
            self.opt_ranges, key_chunk = self.store.forward_chunks(nchunks, lead=True)
            self.engine.set_chunks(key_chunk)
            self.opt_events = [torch.cuda.Event() for _ in self.opt_ranges]
            self.late_event = torch.cuda.Event()
        self.engine.refresh_weights()
        if self.opt_ranges is not None:
            # Seed the pipeline: every chunk event is recorded once (after the initial pack) and pending, so the
            # FIRST step -- possibly the one a StepPlan records -- already issues the forward / backward waits on
            # the optimizer chunks that later replays need (they are trivially satisfied here).
            side = self.engine.side
            plan.wait_stream(side, torch.cuda.current_stream(self.device))
            for ev in self.opt_events:
                plan.record_event(ev, side)
            self.engine._pending = {c: ev for c, ev in enumerate(self.opt_events)}
            if self.engine.pack.late_chunk is not None:
                plan.record_event(self.late_event, side)
                self.engine._pending[self.engine.pack.late_chunk] = self.late_event
        # The optimizer chunks (and the weight-gradient / norm / reducer streams) keep using the persistent buffers
        # after step() returns; marking them used on those streams makes the caching allocator hold their memory until
        # that work has finished when the trainer is dropped (no reuse by a later allocation while a chunk still runs).
        if self.device.type == "cuda":
            streams = list(getattr(self.engine, "sides", None) or [])
            if self.norm_parts is not None:
                streams.append(self.norm_parts.stream)
            if self.reducer is not None and getattr(self.reducer, "stream", None) is not None:
                streams.append(self.reducer.stream)
            bufs = [self.store.params, self.store.grads, self.m, self.v, self.ema, self.state,
                    getattr(getattr(self.engine, "pack", None), "buf", None)]
            for b in bufs:
                if b is not None:
                    for s in streams:
                        b.record_stream(s)

    # ------------------------------------------------------------------------------------------
    def _watermarks(self, tape):
        """Per backward position k: flat offset below which every gradient is final."""
        done_at = {}
        for k in range(len(tape) - 1, -1, -1):  # a label is complete at its earliest tape entry
            done_at[tape[k][1]["label"]] = k
        order = self.store.order
        comp = [done_at.get(param_label(key), 0) for key in order]
        # prefix minimum of completion index over the flat order: prefix final once k <= that value
        marks = []
        run = math.inf
        for key, c in zip(order, comp):
            run = min(run, c)
            marks.append((self.store.offsets[key][0] + self.store.offsets[key][1], run))
        return marks

    def _on_progress(self, tape, k):
        # after finishing entry k (going backwards), every param whose label completed at >= k is final
        marks = self._progress
        upto = 0
        for end, run in marks:
            if run >= k:
                upto = end
            else:
                break
        if self.reducer is not None:
            self.reducer.ready(upto)
        if self.norm_parts is not None:
            self.norm_parts.ready(upto)

    # ------------------------------------------------------------------------------------------
    def step(self, x0, noise, t, text=None, mask=None, mask_keep=None, klass=None):
        """One training step on device tensors: x0/noise (B,4,H,W) fp32, t (B,) int64, text (B,S,C) fp32,
        mask (B,18,MH,MW) fp32 (one-hot), mask_keep (B,) fp32 cond-drop multipliers or None."""
        return self._step(x0, noise, t, text, mask, mask_keep, klass)

    def _step(self, x0, noise, t, text, mask, mask_keep, klass=None):
        eng, st = self.engine, self.store
        B, C, H, W = x0.shape
        xt = torch.empty_like(x0)
        K.add_noise(x0, noise, t, self.sqrt_abar, self.sqrt_1m_abar, xt)
        pred, ctx = eng.forward(xt, t, text, mask, mask_keep=mask_keep, klass=klass)
        dpred = eng.new_dpred(B, H, W)
        eng.loss(pred, noise, dpred, self.state[S_LOSS:S_LOSS + 1], gscale_dev=self.state[S_SCALE:S_SCALE + 1])
        L = _lib.lib()
        if self.world > 1:  # this rank's non-finite-loss flag into the gradient tail (all-reduced with the last bucket)
            _lib.check(L.sdmi_loss_flag(self.state[S_LOSS:].data_ptr(), st.grads[st.numel:].data_ptr(), 0, K._stream()),
                       "sdmi_loss_flag")
        if self.reducer is not None and self.base == "dit":
            self.reducer.reset()
            eng.backward(ctx, dpred, on_progress=self._on_progress_dit)
            self._tail_mark(0)
            self.reducer.finish()
            self._tail_mark(1)
        elif self.reducer is not None:
            self.reducer.reset()
            if self._progress is None:
                self._progress = self._watermarks(ctx["tape"])
            eng.backward(ctx, dpred, on_progress=self._on_progress)
            self._tail_mark(0)
            self.reducer.finish()
            self._tail_mark(1)
        elif self.norm_parts is not None:
            self.norm_parts.reset()
            if self.base == "dit":
                eng.backward(ctx, dpred, on_progress=self._on_progress_dit)
            else:
                if self._progress is None:
                    self._progress = self._watermarks(ctx["tape"])
                eng.backward(ctx, dpred, on_progress=self._on_progress)
        else:
            eng.backward(ctx, dpred)
        hp = self.hp
        # Non-finite loss: the reference skips before scaler.update() (:348-352), leaving the scale alone. N > 1: the
        # all-reduced sum of every rank's flag decides, so all replicas skip together (and keep their scale) when any
        # rank's loss is non-finite; a non-finite gradient norm (all-reduced gradients: identical on every rank) skips
        # and backs the scale off everywhere (:366-371).
        if self.world > 1:
            _lib.check(L.sdmi_loss_flag(st.grads[st.numel:].data_ptr(), self.state[S_DPFLAG:].data_ptr(), 1,
                                        K._stream()), "sdmi_loss_flag")
        if self.norm_parts is not None:
            self.norm_parts.finish(hp["clip"], self.state, hp["growth"], 1, 1.0)
        elif self.red_norm is not None:  # the reducer's per-bucket pieces (all-reduced sums: grad_div = world)
            finalize_norm(self.red_norm, hp["clip"], self.state, hp["growth"], 1 if self.world == 1 else 2,
                          float(self.world))
        else:
            wsb = L.sdmi_optim_workspace_for(st.numel)  # one partial per norm block, any model size
            ws = torch.empty(wsb // 4, dtype=torch.float32, device=self.device)
            _lib.check(L.sdmi_clip_unscale_ws(st.grads.data_ptr(), st.numel, hp["clip"], self.state.data_ptr(),
                                              ws.data_ptr(), wsb, hp["growth"], 1 if self.world == 1 else 2,
                                              float(self.world), K._stream()), "sdmi_clip_unscale_ws")
        ema_decay = hp["ema"] if hp["ema"] is not None else 0.0
        if self.opt_ranges is None:
            _lib.check(L.sdmi_adam_ema_bf16(st.params.data_ptr(), st.grads.data_ptr(), self.m.data_ptr(),
                                            self.v.data_ptr(), K._p(self.ema), st.numel, self.state.data_ptr(), hp["lr"],
                                            hp["b1"], hp["b2"], hp["eps"], ema_decay, 1.0 - ema_decay,
                                            None, K._stream()), "sdmi_adam_ema")
            eng.refresh_weights()
            return self.state
        side = eng.side
        plan.wait_stream(side, torch.cuda.current_stream(self.device))
        with torch.cuda.stream(side):
            for c, (lo, hi) in enumerate(self.opt_ranges):
                e = self.ema[lo:hi] if self.ema is not None else None
                _lib.check(L.sdmi_adam_ema_bf16(st.params[lo:hi].data_ptr(), st.grads[lo:hi].data_ptr(),
                                                self.m[lo:hi].data_ptr(), self.v[lo:hi].data_ptr(), K._p(e), hi - lo,
                                                self.state.data_ptr(), hp["lr"], hp["b1"], hp["b2"], hp["eps"],
                                                ema_decay, 1.0 - ema_decay, None, K._stream()), "sdmi_adam_ema")
                eng.pack.run_chunk(c)
                plan.record_event(self.opt_events[c], side)
            late = eng.pack.late_chunk
            if late is not None:  # backward-only layouts, behind every forward chunk
                eng.pack.run_chunk(late)
                plan.record_event(self.late_event, side)
        eng._pending = {c: ev for c, ev in enumerate(self.opt_events)}
        if late is not None:
            eng._pending[late] = self.late_event
        return self.state

    def measure_exchange_tail(self, on=True):
        """Eager steps record two events on the compute stream: when the backward (every gradient kernel, side streams
        joined) is done and when the last all-reduce bucket has been waited for; their distance is the gradient exchange
        left exposed after the backward (exchange_tail_ms)."""
        self.tail_events = [torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)] if on else None

    def _tail_mark(self, i):
        if self.tail_events is not None:
            self.tail_events[i].record()

    def exchange_tail_ms(self):
        if self.tail_events is None:
            return None
        return self.tail_events[0].elapsed_time(self.tail_events[1])

    def _on_progress_dit(self, i):
        """DiT backward finished layer i: proj_out and layers i..L-1 are final (the flat prefix up to layer i)."""
        if self._dit_marks is None:
            marks = {}
            for key in self.store.order:
                if key.startswith("transformer_layers.") and ".adaptive_norm_layer." not in key:
                    li = int(key.split(".")[1])
                    off, n = self.store.offsets[key]
                    marks[li] = max(marks.get(li, 0), off + n)
            self._dit_marks = marks
        if self.reducer is not None:
            self.reducer.ready(self._dit_marks[i])
        if self.norm_parts is not None:
            self.norm_parts.ready(self._dit_marks[i])

    _dit_marks = None

    def loss(self):
        return self.state[S_LOSS]

    def ema_state_dict(self):
        if self.ema is None:
            raise RuntimeError("this trainer keeps no EMA copy (ema_decay=None)")
        self.sync_optimizer()
        return {k: self._export(self.store.view(self.ema, k)) for k in self.store.order}

    @staticmethod
    def _export(v):
        # GEMM-natural (co, kh, kw, ci) weights are permuted views: hand out contiguous torch-order copies so saved
        # checkpoints match the reference's state dicts (safetensors and .view() consumers need contiguity)
        return v if v.is_contiguous() else v.contiguous()

    def state_dict(self):
        """Model state dict: READ-ONLY snapshots of the flat fp32 master weights, safe to read or save on the current
        stream (it first waits for the chunked optimizer step still in flight on the side stream). Entries are views
        of the master buffer for torch-order weights but contiguous COPIES for the GEMM-natural (co, kh, kw, ci) conv
        weights, so writing into them does not update the model consistently: load weights through the module's
        load_state_dict / sdmi_invalidate path, or a new DDPMTrainer. Never read store.params / store.p directly after
        step() without sync_optimizer()."""
        self.sync_optimizer()
        return {k: self._export(self.store.p[k]) for k in self.store.order}

    def sync_optimizer(self):
        """The current stream waits for the chunked optimizer step still in flight (parameters, EMA and packed
        weights are final for stream-ordered readers afterwards)."""
        need = getattr(self.engine, "_need_all", None)
        if need is not None:
            need()
