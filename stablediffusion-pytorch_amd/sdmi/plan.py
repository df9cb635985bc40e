"""Launch-plan record / replay: the host side of a training step as a flat list of native calls.

One eager step issues ~1,100 kernel launches through the C ABI (plus stream / event edges and, for N > 1, the
RCCL bucket all-reduces); Python + ctypes bookkeeping costs ~15 us per launch, so an eager step is bound by the
host at ~17 ms. A hipGraph removes that cost only for single-stream captures on this ROCm (a two-stream capture
replays at the same ~16 ms of host time), and RCCL collectives sit between segments. StepPlan instead records
the step ONCE -- every libsdmi entry point call with its already-marshalled arguments, every stream / event edge,
every collective -- while running it for real, with all its temporaries allocated from a private memory pool
that stays reserved; replay() re-issues exactly those calls: same pointers, same streams, same ordering, no
Python-side shape logic, ~1 us per call. Per-step inputs live in static buffers filled before each replay.

Hazard model = the eager step's: replay issues the same operations on the same streams in the same order, and
no memory of the pool is handed to anything outside the plan between replays."""
import torch

RECORDING = None  # list of (callable, args) while a plan is being recorded


def record(fn, *args):
    """Call fn(*args) now and, while recording, append it to the plan."""
    r = fn(*args)
    if RECORDING is not None:
        RECORDING.append((fn, args))
    return r


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


def wait_stream(dst, src):
    record(dst.wait_stream, src)


def record_event(ev, stream):
    record(ev.record, stream)


def wait_event(stream, ev):
    record(stream.wait_event, ev)


class StepPlan:
    def __init__(self, step_fn, device=None):
        global RECORDING
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        torch.cuda.synchronize(self.device)
        self.pool = torch.cuda.MemPool()
        ops = []
        with torch.cuda.use_mem_pool(self.pool, device=self.device):
            RECORDING = ops
            try:
                step_fn()
            finally:
                RECORDING = None
        torch.cuda.synchronize(self.device)
        self.ops = ops

    def __len__(self):
        return len(self.ops)

    def replay(self):
        for fn, args in self.ops:
            r = fn(*args)
            # libsdmi entry points return an int status (0 = ok); torch / dist calls return None, tensors or works
            if type(r) is int and r != 0:
                raise RuntimeError(f"plan replay: {getattr(fn, '__name__', fn)} failed with status {r}")
