"""Launch-plan record / replay: the host side of a training step recorded once, re-issued from C++.

One eager step issues ~1,000 kernel launches through the C ABI (plus stream / event edges and, for N > 1, the RCCL
bucket all-reduces). Issued from Python, each launch costs the ctypes marshalling, the library's host-side planning
(descriptor validation, split-K / tile choice) and the HIP launch: ~12 ms of host time per cond-UNet step, as much
as the device time. StepPlan records the step ONCE while running it for real -- libsdmi appends every kernel launch
with a copy of its marshalled arguments to a native plan (csrc/plan.hip), this module notes the stream / event edges
and, as numbered callouts, the work the library does not own (RCCL collectives, torch copies) -- with all
temporaries allocated from a private memory pool that stays reserved. replay() then runs the recorded launches in
C++ (one hipLaunchKernel each: same pointers, grids, streams and order), returning to Python only at callouts.
Per-step inputs live in static buffers refilled before each replay.

Hazard model = the eager step's: replay issues the same operations on the same streams in the same order, and no
memory of the pool is handed to anything outside the plan between replays."""
import ctypes

import torch

RECORDING = None  # callout list [(callable, args)] while a plan is being recorded
KEEP = None       # objects the recorded plan refers to by handle (events) -- kept alive with the plan


def _lib():
    from . import _lib as L
    return L.lib()


def record(fn, *args):
    """Call fn(*args) now and, while recording, make it a callout of the plan (replayed from Python)."""
    r = fn(*args)
    if RECORDING is not None:
        RECORDING.append((fn, args))
        _check(_lib().sdmi_plan_note_callout(len(RECORDING) - 1), "sdmi_plan_note_callout")
    return r


def _check(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed with status {rc}")


def as_operand(t, dtype=torch.float32):
    """t as a contiguous tensor of `dtype` for a raw-pointer kernel argument. When a conversion / copy is needed
    it is a recorded step of its own (a plan replays it, so the kernels never read a stale copy)."""
    if t.dtype == dtype and t.is_contiguous():
        return t
    out = torch.empty(t.shape, dtype=dtype, device=t.device)
    record(out.copy_, t)
    return out


def timesteps(t, device):
    """int64 (n,) device view of a timestep argument (int, 0-d / 1-d tensor, host or device)."""
    if isinstance(t, torch.Tensor) and t.device == torch.device(device) and t.dtype == torch.int64 and t.is_contiguous():
        return t.reshape(-1)
    if isinstance(t, torch.Tensor) and t.device.type == "cuda":
        return as_operand(t.reshape(-1), torch.int64)
    return torch.as_tensor(t, device=device).long().reshape(-1)  # host value: baked into the plan by design


def record_event(ev, stream):
    ev.record(stream)
    if RECORDING is not None:
        KEEP.append(ev)
        _check(_lib().sdmi_plan_note_event(ev.cuda_event, stream.cuda_stream), "sdmi_plan_note_event")


def wait_event(stream, ev):
    stream.wait_event(ev)
    if RECORDING is not None:
        KEEP.append(ev)
        _check(_lib().sdmi_plan_note_wait(stream.cuda_stream, ev.cuda_event), "sdmi_plan_note_wait")


def wait_stream(dst, src):
    """dst waits for everything issued so far on src (an event edge the plan can replay)."""
    if RECORDING is None:
        dst.wait_stream(src)
        return
    ev = torch.cuda.Event()
    record_event(ev, src)
    wait_event(dst, ev)


class StepPlan:
    def __init__(self, step_fn, device=None):
        global RECORDING, KEEP
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        torch.cuda.synchronize(self.device)
        self.pool = torch.cuda.MemPool()
        lib = _lib()
        self.handle = None
        ops, keep = [], []
        with torch.cuda.use_mem_pool(self.pool, device=self.device):
            _check(lib.sdmi_plan_begin(), "sdmi_plan_begin")
            RECORDING, KEEP = ops, keep
            h = ctypes.c_void_p()
            try:
                step_fn()
            finally:
                RECORDING, KEEP = None, None
                _check(lib.sdmi_plan_end(ctypes.byref(h)), "sdmi_plan_end")
                self.handle = h
        torch.cuda.synchronize(self.device)
        self.ops = ops
        self.keep = keep
        self._cid, self._next = ctypes.c_int(0), ctypes.c_int(0)

    def info(self):
        """(recorded ops, kernel launches, callouts)."""
        n, k = ctypes.c_int(0), ctypes.c_int(0)
        _check(_lib().sdmi_plan_info(self.handle, ctypes.byref(n), ctypes.byref(k)), "sdmi_plan_info")
        return n.value, k.value, len(self.ops)

    def __len__(self):
        return self.info()[0]

    def collectives(self):
        """Number of recorded bucket all-reduces: native RCCL ops (sdmi_allreduce) plus torch.distributed callouts."""
        lib = _lib()
        n, kind = self.info()[0], ctypes.c_int(0)
        native = 0
        for i in range(n):
            _check(lib.sdmi_plan_op_info(self.handle, i, ctypes.byref(kind), None, None, None, None), "sdmi_plan_op_info")
            native += kind.value == 4
        return native + sum(1 for fn, _ in self.ops if getattr(fn, "__name__", "") == "_issue")

    def replay(self):
        lib = _lib()
        cid, nxt = self._cid, self._next
        pos = 0
        while True:
            rc = lib.sdmi_plan_replay(self.handle, pos, ctypes.byref(cid), ctypes.byref(nxt))
            if rc != 0:
                raise RuntimeError(f"plan replay failed at op {nxt.value} with status {rc}")
            if cid.value < 0:
                return
            fn, args = self.ops[cid.value]
            fn(*args)
            pos = nxt.value

    def __del__(self):
        if getattr(self, "handle", None) is not None and self.handle.value:
            try:
                _lib().sdmi_plan_destroy(self.handle)
            except Exception:
                pass
            self.handle = None
