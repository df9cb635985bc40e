"""Bucketed, backward-overlapped gradient all-reduce over the flat fp32 gradient buffer.

Replaces DistributedDataParallel's reducer (train_ddpm_cond_celebhq_multi_gpu.py:257-263; 25 MB
buckets, allreduce-then-average) for the HIP trainer: the flat buffer is ordered so the backward
pass finalises it front to back; as soon as a prefix of at least `bucket_bytes` is final it is
all-reduced (SUM) on a dedicated stream while the backward continues. The averaging (1/world) is
folded into the optimizer's unscale/clip coefficient, so no extra pass touches the gradients.
On ROCm the "nccl" backend is RCCL over xGMI; the same class runs with gloo on CPU for tests.

wire="bf16" (off by default; SDMI_GRAD_WIRE=bf16 in the trainer) sends each bucket as bf16: half the bytes on the
xGMI links, at the cost of bf16 rounding of every rank's gradient and of the ring's partial sums (the reference's DDP
averages fp32 gradients). The fp32 buffer is rounded into a bf16 staging copy on the reducer stream, all-reduced,
and widened back once the collective has completed."""
import torch
import torch.distributed as dist

from . import plan


class BucketReducer:
    def __init__(self, flat, group=None, bucket_bytes=64 << 20, wire="fp32"):
        if wire not in ("fp32", "bf16"):
            raise ValueError(f"gradient wire format {wire!r}: fp32 or bf16")
        self.flat = flat
        self.group = group
        self.wire = wire
        self.bucket = max(1, bucket_bytes // flat.element_size())
        self.total = flat.numel()
        self.cuda = flat.is_cuda
        self.stream = torch.cuda.Stream(device=flat.device) if self.cuda else None
        self.producers = []  # extra streams that write gradients (the engine's weight-gradient stream)
        self.reset()

    def reset(self):
        self.launched = 0
        self.works = []

    def _issue(self, view):
        """all-reduce on the reducer stream (also the unit a recorded StepPlan re-issues)."""
        if self.cuda:
            with torch.cuda.stream(self.stream):
                self._issue_on(view)
        else:
            self._issue_on(view)

    def _issue_on(self, view):
        if self.wire == "bf16":
            wire = view.to(torch.bfloat16)
            self.works.append((dist.all_reduce(wire, group=self.group, async_op=True), wire, view))
        else:
            self.works.append((dist.all_reduce(view, group=self.group, async_op=True), None, None))

    def _launch(self, lo, hi):
        view = self.flat[lo:hi]
        if self.cuda:
            for st in [torch.cuda.current_stream(self.flat.device)] + list(self.producers):
                ev = torch.cuda.Event()
                plan.record_event(ev, st)
                plan.wait_event(self.stream, ev)
        plan.record(self._issue, view)

    def ready(self, upto):
        """Gradients at flat offsets < upto are final."""
        while upto - self.launched >= self.bucket:
            hi = self.launched + self.bucket
            self._launch(self.launched, hi)
            self.launched = hi
        if upto >= self.total and self.launched < self.total:
            self._launch(self.launched, self.total)
            self.launched = self.total

    def _drain(self):
        for w, wire, view in self.works:
            w.wait()  # NCCL/RCCL: makes the current stream wait for the collective (no host sync)
            if wire is not None:
                view.copy_(wire)  # widen the summed bf16 bucket back into the fp32 gradients (current stream)
        self.works = []

    def finish(self):
        if self.launched < self.total:
            self.ready(self.total)
        plan.record(self._drain)
        if self.cuda:
            plan.wait_stream(torch.cuda.current_stream(self.flat.device), self.stream)
