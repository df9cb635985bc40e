"""Bucketed, backward-overlapped gradient all-reduce over the flat fp32 gradient buffer.

Replaces DistributedDataParallel's reducer (train_ddpm_cond_celebhq_multi_gpu.py:257-263; 25 MB
buckets, allreduce-then-average) for the HIP trainer: the flat buffer is ordered so the backward
pass finalises it front to back; as soon as a prefix of at least `bucket_bytes` is final it is
all-reduced (SUM) on a dedicated stream while the backward continues. The averaging (1/world) is
folded into the optimizer's unscale/clip coefficient, so no extra pass touches the gradients.
On ROCm the "nccl" backend is RCCL over xGMI; the same class runs with gloo on CPU for tests.

Gradient norm (clip_grad_norm_, :362-365) in the exchange: with `norm` (a NormBlocks), each bucket's block sums of
squares run on the reducer stream as soon as ITS all-reduce has completed -- while the next bucket is on the wire --
so after the last bucket only the last bucket's pieces and the finalisation remain. Buckets are whole numbers of norm
blocks, and a block's partial depends only on its own (all-reduced) data, so the norm is bitwise the whole-buffer norm
(csrc/optim.hip sumsq_block_kernel).

With an "nccl" (RCCL) group on the GPU the bucket all-reduces are issued by the library's own RCCL communicator on
the reducer stream (NativeComm, csrc/comm.hip): no torch.distributed call per bucket, no Python callout in a replayed
plan, and the collective runs on the reducer's hardware queue instead of the process group's internal stream, which
shares a queue with one of the step's compute streams (sdmi/streams.py; SDMI_NATIVE_COMM=0: torch.distributed).

wire="bf16" (off by default; SDMI_GRAD_WIRE=bf16 in the trainer) sends each bucket as bf16: half the bytes on the
xGMI links, at the cost of bf16 rounding of every rank's gradient and of the ring's partial sums (the reference's DDP
averages fp32 gradients). The fp32 bucket is rounded into a persistent bf16 staging buffer by a HIP kernel on the
reducer stream (sdmi_cast_bf16), all-reduced, and widened back by a HIP kernel that also produces the bucket's norm
blocks (sdmi_widen_bf16_sumsq): no aten kernel on the exchange path."""
import ctypes
import math
import os

import torch
import torch.distributed as dist

from . import _lib
from . import plan
from . import streams

CPU_NORM_BLOCK = 1 << 17  # CPU (gloo test) tensors: the same block size as csrc/optim.hip NORM_BLK


class NormBlocks:
    """Partial slots of the gradient sum of squares, one per block of `blk` elements at absolute flat offsets
    [0, numel). launch(g, lo, hi) fills the slots of [lo, hi) (lo on a block boundary; hi on one or == numel)."""

    def __init__(self, numel, device):
        self.device = torch.device(device)
        self.cuda = self.device.type == "cuda"
        if self.cuda:
            from . import _lib
            self.blk = int(_lib.lib().sdmi_norm_block())
        else:
            self.blk = CPU_NORM_BLOCK
        self.numel = numel
        self.n = max(1, math.ceil(numel / self.blk))
        self.partials = torch.zeros(self.n, dtype=torch.float32, device=self.device)

    def floor(self, off):
        return off // self.blk * self.blk

    def _check_range(self, lo, hi):
        hi = min(hi, self.numel)
        assert lo % self.blk == 0 and (hi == self.numel or hi % self.blk == 0), (lo, hi)
        return hi

    def launch(self, g, lo, hi, stream=None):
        hi = self._check_range(lo, hi)
        if hi <= lo:
            return
        dst = self.partials[lo // self.blk:]
        if self.cuda:
            from . import _lib
            _lib.check(_lib.lib().sdmi_sumsq_blocks(g[lo:hi].data_ptr(), hi - lo, dst.data_ptr(),
                                                    (stream or torch.cuda.current_stream(self.device)).cuda_stream),
                       "sdmi_sumsq_blocks")
        else:
            self._cpu_blocks(g[lo:hi], dst)

    def widen(self, wire, g, lo, hi, stream):
        """g[lo:hi] = float(wire[lo:hi]) with the norm blocks of [lo, min(hi, numel)) (bf16 wire, reducer stream)."""
        nh = self._check_range(lo, hi)
        if self.cuda:
            from . import _lib
            L = _lib.lib()
            if nh > lo:
                _lib.check(L.sdmi_widen_bf16_sumsq(wire[lo:nh].data_ptr(), g[lo:nh].data_ptr(), nh - lo,
                                                   self.partials[lo // self.blk:].data_ptr(), stream.cuda_stream),
                           "sdmi_widen_bf16_sumsq")
            if hi > nh:  # the flag tail past numel (not part of the norm)
                _lib.check(L.sdmi_widen_bf16_sumsq(wire[nh:hi].data_ptr(), g[nh:hi].data_ptr(), hi - nh, None,
                                                   stream.cuda_stream), "sdmi_widen_bf16_sumsq")
        else:
            g[lo:hi].copy_(wire[lo:hi])
            if nh > lo:
                self._cpu_blocks(g[lo:nh], self.partials[lo // self.blk:])

    def _cpu_blocks(self, x, dst):
        for b in range(math.ceil(x.numel() / self.blk)):
            v = x[b * self.blk:(b + 1) * self.blk].double()
            dst[b] = float((v * v).sum())

    def whole(self, g):
        """Every block of g[0:numel) at once (the unsplit reference of the pieces)."""
        self.launch(g, 0, self.numel)


def rccl_path():
    """The RCCL shared library torch itself uses (one RCCL in the process), else the system's."""
    p = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
    return p if os.path.exists(p) else "librccl.so"


def agree(ok, group, device):
    """True on every rank iff `ok` holds on every rank of `group` (MIN all-reduce of a flag over the torch group): a
    decision all ranks take together, so no rank waits in a collective its peers have given up on."""
    flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=device)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
    return bool(flag.item())


def allreduce_selfcheck(all_reduce, rank, world, device, n=1031):
    """One-time correctness check of an in-place SUM all-reduce `all_reduce(buf)` (collective: every rank calls it):
    an odd-length fp32 and bf16 bucket whose closed-form sum is exact in both types -- rank r contributes (r + 1) * w_i
    with w_i = 1 + i % 7, the sum is world (world + 1) / 2 * w_i (exact in bf16 up to world 16). A wrong count, dtype,
    buffer or rank mapping shows up at any world size > 1. Returns this rank's verdict (combine it with agree())."""
    w = 1.0 + torch.arange(n, device=device, dtype=torch.float32).remainder(7)
    want = w * (world * (world + 1) / 2)
    ok = True
    for dt in (torch.float32, torch.bfloat16):
        buf = (w * (rank + 1)).to(dt)
        all_reduce(buf)
        ok = ok and bool(torch.equal(buf.float(), want.to(dt).float()))
    return ok


class NativeComm:
    """An RCCL communicator owned by libsdmi over the ranks of `group` (rank 0's unique id broadcast through the
    group), used for in-place SUM all-reduces on a given stream (sdmi_allreduce).

    create() is the collective constructor the reducer uses: every step of the setup that can fail on one rank alone
    (binding librccl, rank 0's unique id, the communicator init) is followed by agree() over the torch group, and the
    finished communicator must pass allreduce_selfcheck() on every rank; otherwise EVERY rank gets None and the
    bucket all-reduces go through torch.distributed on all of them (never a mix, never a rank left waiting)."""

    def __init__(self, handle, rank, world, lib=None):
        self.handle, self.rank, self.world = handle, rank, world
        self.lib = lib or _lib.lib()

    @classmethod
    def create(cls, group, device, lib=None):
        import sys
        lib = lib or _lib.lib()
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        flag_dev = torch.device(device)

        def say(why):
            if rank == 0:
                print(f"sdmi.reducer: library RCCL communicator unavailable ({why}); bucket all-reduces go through "
                      f"torch.distributed on every rank", file=sys.stderr)
            return None

        uid = (ctypes.c_ubyte * 128)()
        try:
            ok = lib.sdmi_comm_load(rccl_path().encode()) == 0
            if ok and rank == 0:
                ok = lib.sdmi_comm_unique_id(uid) == 0
        except Exception:  # noqa: BLE001 -- any local failure becomes this rank's vote
            ok = False
        if not agree(ok, group, flag_dev):
            return say("librccl not bound or no unique id on some rank")
        box = [bytes(uid)]
        dist.broadcast_object_list(box, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
        uid = (ctypes.c_ubyte * 128).from_buffer_copy(box[0])
        h = ctypes.c_void_p()
        cuda = flag_dev.type == "cuda"
        try:
            if cuda:
                with torch.cuda.device(flag_dev):
                    ok = lib.sdmi_comm_init(uid, world, rank, ctypes.byref(h)) == 0 and bool(h.value)
            else:  # (the CPU test of this protocol, with a stand-in library)
                ok = lib.sdmi_comm_init(uid, world, rank, ctypes.byref(h)) == 0 and bool(h.value)
        except Exception:  # noqa: BLE001
            ok = False
        comm = cls(h if ok else None, rank, world, lib)
        if not agree(ok, group, flag_dev):
            comm.close()
            return say("communicator init failed on some rank")
        stream = torch.cuda.current_stream(flag_dev) if cuda else None
        try:
            ok = allreduce_selfcheck(lambda b: comm.all_reduce(b, stream), rank, world, flag_dev)
        except RuntimeError:
            ok = False
        if not agree(ok, group, flag_dev):
            comm.close()
            return say("all-reduce self-check failed on some rank")
        return comm

    def all_reduce(self, buf, stream):
        dt = {torch.float32: 0, torch.bfloat16: 1}[buf.dtype]
        _lib.check(self.lib.sdmi_allreduce(self.handle, buf.data_ptr(), buf.numel(), dt,
                                           stream.cuda_stream if stream is not None else None), "sdmi_allreduce")

    def close(self):
        h = getattr(self, "handle", None)
        if h is not None and h.value:
            try:
                self.lib.sdmi_comm_destroy(h)
            except Exception:  # noqa: BLE001
                pass
        self.handle = None

    def __del__(self):
        import sys
        if not sys.is_finalizing():  # (at exit the process ends the communicator)
            self.close()


class BucketReducer:
    def __init__(self, flat, group=None, bucket_bytes=64 << 20, wire="fp32", norm=None, stream=None):
        if wire not in ("fp32", "bf16"):
            raise ValueError(f"gradient wire format {wire!r}: fp32 or bf16")
        self.flat = flat
        self.group = group
        self.wire = wire
        self.norm = norm
        self.bucket = max(1, bucket_bytes // flat.element_size())
        if norm is not None:  # whole norm blocks per bucket
            self.bucket = max(norm.blk, (self.bucket + norm.blk - 1) // norm.blk * norm.blk)
        self.total = flat.numel()
        self.cuda = flat.is_cuda
        # stream: an existing stream idle during the backward (the engine's context stream) to run on, so the step
        # does not add one more stream to the few hardware queues a process gets
        self.stream = (stream or streams.new_stream(flat.device)) if self.cuda else None
        self.wire_buf = torch.empty(self.total, dtype=torch.bfloat16, device=flat.device) if wire == "bf16" else None
        self.producers = []  # extra streams that write gradients (the engine's weight-gradient stream)
        self.comm = None
        if self.cuda and dist.get_backend(group) == "nccl" and os.environ.get("SDMI_NATIVE_COMM", "1") != "0":
            # collective decision (NativeComm.create): every rank gets the library communicator, or none does
            self.comm = NativeComm.create(group, flat.device)
        self.reset()

    def reset(self):
        self.launched = 0
        self.works = {}    # bucket index -> (work, lo, hi), issued and not yet waited for
        self.pending = []  # bucket indices in issue order whose completion work is not yet queued
        self.nb = 0

    def _issue(self, i, lo, hi):
        """all-reduce of bucket i on the reducer stream (the unit a recorded StepPlan re-issues as a callout)."""
        if self.comm is not None:
            self.comm.all_reduce(self.wire_buf[lo:hi] if self.wire == "bf16" else self.flat[lo:hi], self.stream)
            return
        if self.cuda:
            with torch.cuda.stream(self.stream):
                self._issue_on(i, lo, hi)
        else:
            self._issue_on(i, lo, hi)

    def _issue_on(self, i, lo, hi):
        buf = self.wire_buf[lo:hi] if self.wire == "bf16" else self.flat[lo:hi]
        self.works[i] = (dist.all_reduce(buf, group=self.group, async_op=True), lo, hi)

    def _wait(self, i):
        """the reducer stream waits for bucket i's collective (NCCL/RCCL: a stream wait, no host sync)."""
        w = self.works.pop(i)[0]
        if self.cuda:
            with torch.cuda.stream(self.stream):
                w.wait()
        else:
            w.wait()

    def _complete(self, i, lo, hi):
        """after bucket i's all-reduce: widen (bf16 wire) and the bucket's norm blocks, on the reducer stream."""
        if self.comm is None:  # (native: the collective ran on the reducer stream itself)
            plan.record(self._wait, i)
        if self.wire == "bf16":
            if self.norm is not None:
                self.norm.widen(self.wire_buf, self.flat, lo, hi, self.stream)
            elif self.cuda:
                from . import _lib
                _lib.check(_lib.lib().sdmi_widen_bf16_sumsq(self.wire_buf[lo:hi].data_ptr(), self.flat[lo:hi].data_ptr(),
                                                            hi - lo, None, self.stream.cuda_stream),
                           "sdmi_widen_bf16_sumsq")
            else:
                self.flat[lo:hi].copy_(self.wire_buf[lo:hi])
        elif self.norm is not None:
            self.norm.launch(self.flat, lo, hi, self.stream)

    def _launch(self, lo, hi):
        if self.cuda:
            for st in [torch.cuda.current_stream(self.flat.device)] + list(self.producers):
                ev = torch.cuda.Event()
                plan.record_event(ev, st)
                plan.wait_event(self.stream, ev)
        if self.wire == "bf16":  # round the final fp32 bucket into the staging buffer on the reducer stream
            if self.cuda:
                from . import _lib
                _lib.check(_lib.lib().sdmi_cast_bf16(self.flat[lo:hi].data_ptr(), self.wire_buf[lo:hi].data_ptr(),
                                                     hi - lo, self.stream.cuda_stream), "sdmi_cast_bf16")
            else:
                self.wire_buf[lo:hi].copy_(self.flat[lo:hi])
        i = self.nb
        self.nb += 1
        if self.comm is not None:  # recorded into a plan by the library itself
            if plan.KEEP is not None:  # the plan's native op holds the raw communicator: keep its owner alive with it
                plan.KEEP.append(self.comm)
            self._issue(i, lo, hi)
        else:
            plan.record(self._issue, i, lo, hi)
        # the previous bucket completes behind this one's issue, so its widening / norm overlaps this collective
        while self.pending:
            j, jlo, jhi = self.pending.pop(0)
            self._complete(j, jlo, jhi)
        self.pending.append((i, lo, hi))

    def ready(self, upto):
        """Gradients at flat offsets < upto are final."""
        while upto - self.launched >= self.bucket:
            hi = self.launched + self.bucket
            self._launch(self.launched, hi)
            self.launched = hi
        if upto >= self.total and self.launched < self.total:
            self._launch(self.launched, self.total)
            self.launched = self.total

    def finish(self):
        if self.launched < self.total:
            self.ready(self.total)
        while self.pending:
            j, jlo, jhi = self.pending.pop(0)
            self._complete(j, jlo, jhi)
        if self.cuda:
            plan.wait_stream(torch.cuda.current_stream(self.flat.device), self.stream)
