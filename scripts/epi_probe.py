"""Epilogue-cost probe for the short-K GEMMs: the same GEMM timed plain, with a bias, with a residual addend and with
a per-sample row bias (back-to-back launches, device time per launch), plus the HBM bytes each form moves, so the
epilogue's share of a latency-bound launch is visible. Usage: python scripts/epi_probe.py"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "stablediffusion-pytorch_amd"))
import torch  # noqa: E402

from sdmi import kernels as K  # noqa: E402


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
    shapes = [(32768, 384, 384), (32768, 1152, 384), (8192, 512, 512), (2048, 768, 768), (512, 512, 512),
              (8192, 288, 288), (8192, 864, 288), (8192, 1152, 288), (8192, 288, 1152)]
    for (M, N, Kd) in shapes:
        x, w = rnd(M, Kd), rnd(N, Kd)
        out, res = torch.empty(M, N, device=dev, dtype=torch.bfloat16), rnd(M, N)
        bias = torch.rand(N, device=dev)
        rb = rnd(32, N)
        t0 = timeit(lambda: K.linear(x, w, out))
        t1 = timeit(lambda: K.linear(x, w, out, bias=bias))
        t2 = timeit(lambda: K.linear(x, w, out, bias=bias, resid=res))
        t3 = timeit(lambda: K.linear(x, w, out, bias=bias, rowbias=rb, rb_mod=32))
        ref = (x.float() @ w.float().t() + bias + res.float())
        K.linear(x, w, out, bias=bias, resid=res)
        err = (out.float() - ref).abs().max().item()
        mb = (M * Kd + N * Kd + M * N) * 2 / 1e6
        print(f"M={M:6d} N={N:5d} K={Kd:5d}  plain {t0:6.1f} us  +bias {t1:6.1f}  +bias+resid {t2:6.1f}  "
              f"+bias+rowbias {t3:6.1f}   {mb:6.1f} MB plain -> {mb / t0:5.2f} TB/s   "
              f"{2 * M * N * Kd / t0 / 1e6:6.1f} TF   max|err| {err:.3g}", flush=True)


if __name__ == "__main__":
    main()
