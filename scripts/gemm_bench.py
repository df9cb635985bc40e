"""Micro-benchmark of the sdmi GEMM family on shapes from the CelebHQ cond-UNet step (B=32, 32x32
latents). The mainloop variant is chosen by SDMI_GEMM_VARIANT (0 register-staged, 2/3 LDS-DMA ring);
run once per variant and compare. Prints one line per shape: name, TFLOP/s, microseconds."""
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
    bf = torch.bfloat16
    out = []
    g = torch.Generator(device=dev).manual_seed(0)

    def rnd(*shape):
        return torch.randn(*shape, device=dev, generator=g).to(bf)

    # 3x3 convs
    for (B, H, C) in ((32, 32, 384), (32, 16, 512), (32, 8, 768)):
        x = rnd(B * H * H, C)
        w = rnd(C, 9 * C)
        y = torch.empty(B * H * H, C, device=dev, dtype=bf)
        us = timeit(lambda: K.conv_fwd(x, B, H, H, C, C, w, C, 3, 3, 1, 1, y, C))
        fl = 2 * B * H * H * C * 9 * C
        out.append((f"conv3x3 fwd {B}x{H}x{H}x{C}", fl / us / 1e6, us))
        dw = torch.empty(C, 9 * C, device=dev)
        us = timeit(lambda: K.conv_wgrad(y, C, x, B, H, H, C, C, C, 3, 3, 1, 1, dw, H, H))
        out.append((f"conv3x3 wgrad {B}x{H}x{H}x{C}", fl / us / 1e6, us))
    # linear (qkv projection) and a square GEMM
    for (M, N, Kd) in ((32768, 1152, 384), (8192, 1536, 512), (4096, 4096, 4096)):
        a = rnd(M, Kd)
        w = rnd(N, Kd)
        c = torch.empty(M, N, device=dev, dtype=bf)
        us = timeit(lambda: K.gemm(M, N, Kd, a, _lib.A_ROWMAJOR, Kd, w, _lib.B_NK, Kd, c, N))
        out.append((f"gemm NK {M}x{N}x{Kd}", 2 * M * N * Kd / us / 1e6, us))
    v = os.environ.get("SDMI_GEMM_VARIANT", "2")
    for name, tf, us in out:
        print(f"v{v} {name:34s} {tf:7.1f} TF {us:9.1f} us")


if __name__ == "__main__":
    main()
