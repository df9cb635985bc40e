"""Captured training step: the reference's step (train_ddpm_cond_celebhq_multi_gpu.py:299-378 /
Model_DiT_12L_train.py:300-375) recorded once and replayed every iteration.

mode "plan" (default): sdmi.plan.StepPlan -- the step's native calls (every libsdmi launch, stream / event edge
and RCCL bucket all-reduce) replayed from a flat list, keeping the two-stream weight-gradient overlap and the
backward-overlapped gradient all-reduce (N > 1), with all temporaries in a private pool.
mode "graph": one hipGraph (torch.cuda.CUDAGraph); single-stream only (a two-stream hipGraph replays at the
same host cost as eager issue on this ROCm) and N == 1 only.
Per-step randomness (noise, t, cond-drop) is drawn into static buffers before each replay, as the reference draws it
per step (one fused HIP launch, sdmi_step_draw)."""
import torch

from .plan import StepPlan


class CapturedTrainStep:
    def __init__(self, trainer, x0, text, empty_text, mask, B, *, warmup=2, generator=None, drop_p=0.1,
                 text_drop_p=0.1, mode="plan"):
        self.tr = trainer
        dev = x0.device
        self.x0, self.text, self.empty, self.mask = x0, text, empty_text, mask
        self.B = B
        self.gen = generator
        self.drop_p, self.text_drop_p = drop_p, text_drop_p
        self.noise = torch.empty_like(x0)
        self.t = torch.empty(B, dtype=torch.long, device=dev)
        self.txt = torch.empty_like(text) if text is not None else None
        self.keep = torch.empty(B, dtype=torch.float32, device=dev)
        self.mode = mode
        self.seed = self.draw_seed(generator)
        self.draws = 0
        self._draw()
        for _ in range(warmup):  # allocator / lazy init outside the recording
            self._run()
        torch.cuda.synchronize(dev)
        if mode == "plan":
            self.plan = StepPlan(self._run, dev)
        elif mode == "graph":
            s = torch.cuda.Stream(device=dev)
            s.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(s):
                self._run()
            torch.cuda.current_stream(dev).wait_stream(s)
            torch.cuda.synchronize(dev)
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph):
                self._run()
            torch.cuda.synchronize(dev)
        else:
            raise ValueError(mode)

    @staticmethod
    def draw_seed(generator=None):
        """The Philox key of this captured step's draws, taken FROM the generator (its state advances, so a rebuilt
        CapturedTrainStep -- resume, per-epoch rebuild -- draws a new sequence, as the reference's per-step torch draws
        would). Without a generator: torch's default generator, with the rank mixed in so DP ranks draw different
        noise / t / cond-drop, as the reference's per-process RNG does (train_seed + rank)."""
        dev = generator.device if generator is not None else torch.device("cpu")
        seed = int(torch.randint(0, 1 << 62, (1,), generator=generator, device=dev).item())
        if generator is None and torch.distributed.is_available() and torch.distributed.is_initialized():
            seed ^= (torch.distributed.get_rank() + 1) * 0x9E3779B97F4A7C15 & ((1 << 62) - 1)
        return seed

    def _run(self):
        self.tr.step(self.x0, self.noise, self.t, self.txt, self.mask, mask_keep=self.keep)

    def _draw(self):
        """One launch (sdmi_step_draw: Philox keyed by the step's seed, a host draw counter as the offset) instead of
        torch's five RNG calls + where (~0.13 ms of the step on the compute stream)."""
        from . import _lib
        txt = self.txt
        if txt is not None:
            assert self.text.is_contiguous() and self.empty.is_contiguous() and txt.is_contiguous()
            assert self.text.dtype == torch.float32 and self.empty.numel() * self.B == self.text.numel()
        _lib.check(_lib.lib().sdmi_step_draw(
            self.noise.data_ptr(), self.noise.numel(), self.t.data_ptr(), self.B, self.tr.num_timesteps,
            self.text.data_ptr() if txt is not None else None, self.empty.data_ptr() if txt is not None else None,
            txt.data_ptr() if txt is not None else None, self.empty.numel() if txt is not None else 0,
            self.text_drop_p, self.keep.data_ptr() if self.mask is not None else None, self.drop_p, self.seed,
            self.draws, torch.cuda.current_stream(self.t.device).cuda_stream), "sdmi_step_draw")
        self.draws += 1

    def step(self):
        self._draw()
        if self.mode == "plan":
            self.plan.replay()
        else:
            self.graph.replay()
