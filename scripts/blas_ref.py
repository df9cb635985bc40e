"""The step's forward-type GEMM shapes (out[M,N] = x[M,K] . w[N,K]^T, bf16 in, bf16 out) through the library
(K.linear, tuned table) and through torch.nn.functional.linear (hipBLASLt), back to back, same inputs: how far the
library's kernels are from the vendor library on the small-K DiT-12L shapes and the UNet's small levels."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "stablediffusion-pytorch_amd"))
import torch  # noqa: E402

from sdmi import kernels as K  # noqa: E402

SHAPES = [  # (label, M, N, K)
    ("dit fc1", 8192, 1152, 288), ("dit fc2", 8192, 288, 1152), ("dit proj", 8192, 288, 288),
    ("dit qkv", 8192, 864, 288), ("dit qkv dgrad", 8192, 288, 864),
    ("unet 32^2 1x1", 32768, 384, 384), ("unet 32^2 fc", 32768, 1152, 384), ("unet 16^2 lin", 8192, 512, 512),
    ("unet 8^2 lin", 2048, 768, 768), ("unet 4^2 lin", 512, 512, 512),
]


def timeit(fn, iters=50):
    for _ in range(5):
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
    for (name, M, N, Kd) in SHAPES:
        x = torch.randn(M, Kd, device=dev, generator=g).bfloat16()
        w = torch.randn(N, Kd, device=dev, generator=g).bfloat16()
        y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        ours = timeit(lambda: K.linear(x, w, y))
        ref = torch.nn.functional.linear(x, w)
        err = (y.float() - ref.float()).abs().max().item()
        blas = timeit(lambda: torch.nn.functional.linear(x, w))
        fl = 2.0 * M * N * Kd
        print(f"{name:14s} M={M:6d} N={N:5d} K={Kd:5d}  sdmi {ours:7.2f} us {fl / ours / 1e6:7.1f} TF   "
              f"hipBLASLt {blas:7.2f} us {fl / blas / 1e6:7.1f} TF   max|diff| {err:.3g}", flush=True)


if __name__ == "__main__":
    main()
