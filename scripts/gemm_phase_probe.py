"""Where the time of one GEMM launch goes, per workgroup: the probe build of the library (python
stablediffusion-pytorch_amd/sdmi/_build.py --trace -> libsdmi_trace.so, loaded through SDMI_LIB_PATH) stamps
s_memrealtime (100 MHz) at kernel entry, when the first k-tile has landed, at the end of the main loop and at the end of
the epilogue of every LDS-DMA workgroup. Prints per shape: launch span (first entry -> last exit), how the workgroups'
entries spread (dispatch ramp / second wave), and the median / p90 prologue, main-loop and epilogue times.
Usage: SDMI_LIB_PATH=.../libsdmi_trace.so python scripts/gemm_phase_probe.py"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "stablediffusion-pytorch_amd"))
import torch  # noqa: E402

from sdmi import kernels as K, _lib  # noqa: E402

SHAPES = [  # (label, M, N, K, epilogue) of out = x[M,K] . w[N,K]^T (+ bias, + residual, SiLU)
    ("dit fc1", 8192, 1152, 288, ""), ("dit fc1 +b", 8192, 1152, 288, "b"), ("dit fc2 +b+r", 8192, 288, 1152, "br"),
    ("dit proj", 8192, 288, 288, ""), ("dit qkv +b", 8192, 864, 288, "b"),
    ("unet 32^2 1x1", 32768, 384, 384, ""), ("unet 32^2 1x1 +b+r", 32768, 384, 384, "br"),
    ("unet 32^2 fc +b", 32768, 1152, 384, "b"), ("unet 16^2 lin +b", 8192, 512, 512, "b"),
    ("unet 8^2 lin +b+s", 2048, 768, 768, "bs"), ("unet 4^2 lin", 512, 512, 512, ""),
]


def main():
    cdll = _lib.lib()._cdll
    cdll.sdmi_gemm_trace_copy.argtypes = [ctypes.c_void_p, ctypes.c_longlong]
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    buf = np.zeros(8 << 16, dtype=np.uint64)
    for (name, M, N, Kd, ep) in SHAPES:
        x = torch.randn(M, Kd, device=dev, generator=g).bfloat16()
        w = torch.randn(N, Kd, device=dev, generator=g).bfloat16()
        y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        kw = {}
        if "b" in ep:
            kw["bias"] = torch.randn(N, device=dev, generator=g)
        if "r" in ep:
            kw["resid"] = torch.randn(M, N, device=dev, generator=g).bfloat16()
        if "s" in ep:
            kw["act"] = 1
        for _ in range(5):
            K.linear(x, w, y, **kw)
        torch.cuda.synchronize()
        assert cdll.sdmi_gemm_trace_clear() == 0
        K.linear(x, w, y, **kw)
        assert cdll.sdmi_gemm_trace_copy(buf.ctypes.data, buf.size) == 0
        t = buf.reshape(-1, 8).astype(np.int64)
        t = t[t[:, 0] > 0]
        if len(t) == 0:
            print(f"{name}: no LDS-DMA workgroups traced")
            continue
        t0 = t[:, 0].min()
        ent, land, loop, done, synced, epi0 = (t[:, i] - t0 for i in range(6))
        span = done.max()
        us = 0.01  # 100 MHz ticks -> us
        q = lambda a, p: float(np.percentile(a, p)) * us  # noqa: E731
        fl = 2.0 * M * N * Kd
        print(f"{name:18s} M={M:6d} N={N:5d} K={Kd:5d} wgs={len(t):5d} span {span * us:6.2f} us ({fl / (span * us) / 1e6:6.1f} TF)"
              f" | entry p50 {q(ent, 50):5.2f} p90 {q(ent, 90):5.2f} max {ent.max() * us:5.2f}"
              f" | first tile p50 {q(land - ent, 50):5.2f} p90 {q(land - ent, 90):5.2f}"
              f" | loop p50 {q(loop - land, 50):5.2f} p90 {q(loop - land, 90):5.2f}"
              f" | epilogue p50 {q(done - loop, 50):5.2f} p90 {q(done - loop, 90):5.2f}"
              f" (wave skew p50 {q(synced - loop, 50):5.2f}, args {q(epi0 - synced, 50):5.2f}, stores {q(done - epi0, 50):5.2f})"
              f" | last exit - last entry {(done.max() - ent.max()) * us:5.2f}", flush=True)


if __name__ == "__main__":
    main()
