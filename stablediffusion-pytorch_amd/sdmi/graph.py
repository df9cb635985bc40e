"""hipGraph capture of the whole training step.

One eager training step issues ~1,100 kernel launches through ctypes; on MI355X the GPU finishes
many of them faster than Python can enqueue them. The step is therefore captured once into a
hipGraph (torch.cuda.CUDAGraph is hipGraph on ROCm) and replayed: every launch, every temporary
(allocated from the graph's private pool) and every pointer is fixed at capture time. Per-step
randomness (noise, t, cond-drop) is drawn into static input buffers before each replay, exactly as
the reference draws it per step (train_ddpm_cond_celebhq_multi_gpu.py:309-342)."""
import torch


class CapturedTrainStep:
    def __init__(self, trainer, x0, text, empty_text, mask, B, *, warmup=2, generator=None, drop_p=0.1,
                 text_drop_p=0.1):
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
        self._draw()
        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):  # warm the allocator / lazy init outside the capture
            for _ in range(warmup):
                self.tr.step(self.x0, self.noise, self.t, self.txt, self.mask, mask_keep=self.keep)
        torch.cuda.current_stream(dev).wait_stream(s)
        torch.cuda.synchronize(dev)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.tr.step(self.x0, self.noise, self.t, self.txt, self.mask, mask_keep=self.keep)
        torch.cuda.synchronize(dev)

    def _draw(self):
        g = self.gen
        self.noise.normal_(generator=g)
        self.t.random_(0, self.tr.num_timesteps, generator=g)
        if self.txt is not None:
            drop = torch.rand(self.B, device=self.t.device, generator=g) < self.text_drop_p  # diffusion_utils.py:21-28
            torch.where(drop[:, None, None], self.empty, self.text, out=self.txt)
        self.keep.copy_((torch.rand(self.B, device=self.t.device, generator=g) > self.drop_p).float())

    def step(self):
        self._draw()
        self.graph.replay()
