"""Streams for the step's concurrent chains, bound to distinct hardware queues on purpose.

HIP gives a process GPU_MAX_HW_QUEUES (4) hardware queues. A stream is bound to one when it is first used: a new
queue while fewer than four exist, then the existing ones in rotation (scripts/queue_probe.py,
profiles/r05_stream_queues.txt). Two busy streams on one queue run one after the other, so which streams share
depends on the first-use order of every stream in the process, RCCL's and torch's included. With an RCCL group
initialised before the engines (the data-parallel path) the first weight-gradient stream landed on the compute
stream's queue and lost its overlap with the backward (+2.1 ms per cond-UNet step).

More queues are no way out: streams on a fifth hardware queue (GPU_MAX_HW_QUEUES=8, or a CU-masked stream, which
always opens a queue of its own) made the step 2.5x slower. So reserve() binds the engines' streams first, while
the process has fewer than four queues: the null stream (the step's main chain), then each reserved stream, every
one on a new queue. Streams bound later (RCCL's) share the four; the engines take the reserved ones in order.
reserve() is called before torch.distributed / RCCL initialisation (bench.py does); without it the engines make
their streams as before."""
import torch

_RESERVED = {}  # device index -> [streams not yet taken]

# streams each bench workload's step takes through new_stream(), in order. UNet trainer: weight-gradient A / B and the
# context stream (which also carries the norm pieces or the reducer). DiT trainer: one weight-gradient side stream, then
# the norm-piece stream (N = 1) or the reducer stream (N > 1). VQVAE trainer: one side stream. Inference workloads
# (vqvae, sample) run on the null stream only. Reserving more than a workload takes would leave a reserved stream
# holding one of the four hardware queues, and RCCL's streams would then rotate onto the step's own queues.
WORKLOAD_STREAMS = {"cond-unet": 3, "uncond-unet": 3, "dit": 2, "vqvae-train": 1, "vqvae": 0, "sample": 0}


def workload_streams(workload, world=1):
    n = WORKLOAD_STREAMS.get(workload, 3)
    return n + 1 if workload == "vqvae-train" and world > 1 else n  # + its bucket reducer's stream


def reserve(device, n=3):
    """First-use the null stream and n fresh streams on `device`, in that order (call before RCCL initialises)."""
    device = torch.device(device)
    if device.type != "cuda":
        return
    idx = device.index if device.index is not None else torch.cuda.current_device()
    with torch.cuda.device(idx):
        torch.empty(1, device=device).zero_()
        got = _RESERVED.setdefault(idx, [])
        for _ in range(n):
            s = torch.cuda.Stream(device=device)
            with torch.cuda.stream(s):
                torch.empty(1, device=device).zero_()
            got.append(s)
        torch.cuda.synchronize(device)


def new_stream(device):
    """A reserved stream of `device` if one is left, else a fresh one."""
    device = torch.device(device)
    idx = device.index if device.index is not None else torch.cuda.current_device()
    got = _RESERVED.get(idx)
    if got:
        return got.pop(0)
    return torch.cuda.Stream(device=device)
