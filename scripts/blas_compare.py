"""Plain-GEMM comparison: sdmi_gemm vs torch.matmul (hipBLASLt) on the step's linear-layer shapes, GPU time by
HIP events over back-to-back launches. Usage: python scripts/blas_compare.py"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "stablediffusion-pytorch_amd"))
import torch  # noqa: E402

from sdmi import kernels as K, _lib  # noqa: E402


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
    bf = torch.bfloat16
    # (M, N, K, kind): nk = y = x W^T (forward), kn = dx = dy W (dgrad), wg = dW = dy^T x (fp32 out)
    for (M, N, Kd, kind) in ((32768, 384, 384, "nk"), (32768, 1152, 384, "nk"), (32768, 384, 384, "kn"),
                             (32768, 384, 1152, "kn"), (2048, 768, 768, "nk"), (2048, 768, 768, "kn"),
                             (8192, 512, 512, "nk"), (384, 384, 32768, "wg"), (1152, 384, 32768, "wg"),
                             (768, 768, 2048, "wg"), (512, 512, 8192, "wg"), (128, 128, 32768, "wg")):
        if kind == "nk":
            a, w = torch.randn(M, Kd, device=dev).to(bf), torch.randn(N, Kd, device=dev).to(bf)
            c = torch.empty(M, N, device=dev, dtype=bf)
            ours = lambda: K.gemm(M, N, Kd, a, _lib.A_ROWMAJOR, Kd, w, _lib.B_NK, Kd, c, N)  # noqa: E731
            theirs = lambda: torch.matmul(a, w.t(), out=c)  # noqa: E731
        elif kind == "kn":
            a, w = torch.randn(M, Kd, device=dev).to(bf), torch.randn(Kd, N, device=dev).to(bf)
            c = torch.empty(M, N, device=dev, dtype=bf)
            ours = lambda: K.gemm(M, N, Kd, a, _lib.A_ROWMAJOR, Kd, w, _lib.B_KN, N, c, N)  # noqa: E731
            theirs = lambda: torch.matmul(a, w, out=c)  # noqa: E731
        else:
            at, b = torch.randn(Kd, M, device=dev).to(bf), torch.randn(Kd, N, device=dev).to(bf)
            c = torch.empty(M, N, device=dev, dtype=torch.float32)
            ours = lambda: K.gemm(M, N, Kd, at, _lib.A_COLMAJOR, M, b, _lib.B_KN, N, c, N)  # noqa: E731
            c16 = torch.empty(M, N, device=dev, dtype=bf)
            theirs = lambda: torch.matmul(at.t(), b, out=c16)  # noqa: E731
        t1, t2 = timeit(ours), timeit(theirs)
        fl = 2 * M * N * Kd
        print(f"{kind} M={M:6d} N={N:5d} K={Kd:6d}: sdmi {t1:7.1f} us ({fl / t1 / 1e6:6.1f} TF)  "
              f"hipBLASLt {t2:7.1f} us ({fl / t2 / 1e6:6.1f} TF)", flush=True)


if __name__ == "__main__":
    main()
