"""Which hardware queue a HIP stream lands on, by creation / first-use order (run under rocprofv3 --kernel-trace and
read Stream_Id / Queue_Id): torch pool streams in creation order and in reverse first-use order, the same after an RCCL
group of one is initialised, and streams made with hipExtStreamCreateWithCUMask (full mask). Each case tags its
streams with a fill of a distinct size so the trace can be decoded. Usage: python scripts/queue_probe.py <case>"""
import ctypes
import os
import socket
import sys

import torch


def tag(stream, n):
    with torch.cuda.stream(stream):
        torch.empty(n, dtype=torch.uint8, device="cuda").fill_(1)
    torch.cuda.synchronize()


_HIP = None
_CUMASK = []  # raw hipStream_t handles this probe created (destroyed by release_cumask_streams)


def cu_mask_stream():
    global _HIP
    hip = _HIP = _HIP or ctypes.CDLL("libamdhip64.so")
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    words = (ncu + 31) // 32
    mask = (ctypes.c_uint32 * words)(*([0xFFFFFFFF] * words))
    s = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), ctypes.c_uint32(words), mask)
    assert rc == 0, rc
    _CUMASK.append(s.value)
    return torch.cuda.ExternalStream(s.value)


def release_cumask_streams(ss):
    """Round-5 finding (gpurun_out/qp_cumask.log: SIGSEGV in __cxa_finalize after the profiler's finalisation): the
    CU-masked streams were foreign hipStream_t's wrapped in torch.cuda.ExternalStream and never destroyed, so static
    teardown ran with them -- and caching-allocator blocks recorded on them -- still live. Drain them, drop every
    torch reference and the allocator's cached blocks, then hipStreamDestroy each one while the runtime is intact."""
    import gc
    for s in ss:
        s.synchronize()
    torch.cuda.synchronize()
    ss.clear()
    gc.collect()
    torch.cuda.empty_cache()
    while _CUMASK:
        rc = _HIP.hipStreamDestroy(ctypes.c_void_p(_CUMASK.pop()))
        assert rc == 0, rc


def main():
    case = sys.argv[1]
    torch.cuda.set_device(0)
    torch.empty(1, device="cuda").fill_(0)  # null stream first
    torch.cuda.synchronize()
    if case.startswith("rccl"):
        import torch.distributed as dist
        sk = socket.socket()
        sk.bind(("127.0.0.1", 0))
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(sk.getsockname()[1]))
        sk.close()
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
        x = torch.ones(1 << 20, device="cuda")
        dist.all_reduce(x)
        torch.cuda.synchronize()
    if case.endswith("cumask"):
        ss = [cu_mask_stream() for _ in range(4)]
    else:
        ss = [torch.cuda.Stream() for _ in range(6)]
    order = list(range(len(ss)))
    if case.endswith("reverse"):
        order.reverse()
    for i in order:
        tag(ss[i], 4096 * (i + 1))
        print(f"stream {i} tagged with fill of {4096 * (i + 1)} bytes", flush=True)
    if case.startswith("rccl"):
        import torch.distributed as dist
        with torch.cuda.stream(ss[0]):
            dist.all_reduce(x)
        torch.cuda.synchronize()
        dist.destroy_process_group()
    if case.endswith("cumask"):
        release_cumask_streams(ss)
        print("cu-masked streams destroyed", flush=True)


if __name__ == "__main__":
    main()
