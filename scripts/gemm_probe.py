"""Probe GEMM efficiency on variants of the dominant conv shape: plain vs implicit-conv A, full vs partial
grid waves. Prints TF/s per variant."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "stablediffusion-pytorch_amd"))
import torch  # noqa: E402

from sdmi import kernels as K, _lib  # noqa: E402


def timeit(fn, iters=30):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    rnd = lambda *s: (torch.rand(*s, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)  # noqa: E731
    for (M, N, Kd) in ((32768, 384, 3456), (32768, 512, 3456), (32768, 256, 3456), (4096, 4096, 4096),
                       (43690, 384, 3456), (16384, 384, 3456), (65536, 384, 3456)):
        a, w = rnd(M, Kd), rnd(N, Kd)
        c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        us = timeit(lambda: K.gemm(M, N, Kd, a, _lib.A_ROWMAJOR, Kd, w, _lib.B_NK, Kd, c, N))
        print(f"plain  M={M:6d} N={N:5d} K={Kd:5d}  {2 * M * N * Kd / us / 1e6:7.1f} TF  {us:8.1f} us", flush=True)
    for (M, N, Kd, mode) in ((32768, 1152, 384, "nk"), (32768, 384, 384, "nk"), (32768, 384, 1152, "kn"),
                             (32768, 384, 384, "kn"), (8192, 1536, 512, "nk"), (8192, 512, 1536, "kn")):
        a = rnd(M, Kd)
        c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        if mode == "nk":
            w = rnd(N, Kd)
            us = timeit(lambda: K.gemm(M, N, Kd, a, _lib.A_ROWMAJOR, Kd, w, _lib.B_NK, Kd, c, N))
        else:
            w = rnd(Kd, N)
            us = timeit(lambda: K.gemm(M, N, Kd, a, _lib.A_ROWMAJOR, Kd, w, _lib.B_KN, N, c, N))
        print(f"linear {mode} M={M:6d} N={N:5d} K={Kd:5d}  {2 * M * N * Kd / us / 1e6:7.1f} TF  {us:8.1f} us", flush=True)
    for (B, H, C, Co) in ((32, 32, 384, 384), (32, 32, 384, 512), (32, 32, 384, 256), (64, 32, 384, 384)):
        x = rnd(B * H * H, C)
        w = rnd(Co, 9 * C)
        y = torch.empty(B * H * H, Co, device=dev, dtype=torch.bfloat16)
        us = timeit(lambda: K.conv_fwd(x, B, H, H, C, C, w, Co, 3, 3, 1, 1, y, Co))
        fl = 2 * B * H * H * Co * 9 * C
        print(f"conv   B={B} {H}x{H} {C}->{Co}        {fl / us / 1e6:7.1f} TF  {us:8.1f} us", flush=True)


if __name__ == "__main__":
    main()
