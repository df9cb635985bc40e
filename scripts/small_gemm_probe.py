"""Small / short-K GEMMs of the step (attention projections, 1x1 convs, low-resolution levels): time per
mainloop variant and split count. Usage: SDMI_GEMM_VARIANT=2|3 python scripts/small_gemm_probe.py"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "stablediffusion-pytorch_amd"))
import torch  # noqa: E402

from sdmi import kernels as K, _lib  # noqa: E402

SHAPES = ((2048, 768, 768, "nk"), (2048, 768, 768, "kn"), (2048, 2304, 768, "nk"), (2048, 384, 384, "nk"),
          (8192, 512, 512, "nk"), (8192, 512, 512, "kn"), (512, 512, 512, "nk"), (512, 512, 512, "kn"),
          (2464, 512, 1024, "nk"), (8192, 256, 256, "nk"), (32768, 384, 384, "nk"), (32768, 384, 384, "kn"))


def timeit(fn, iters=20):
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
    for (M, N, Kd, mode) in SHAPES:
        a = rnd(M, Kd)
        c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        if mode == "nk":
            w = rnd(N, Kd)
            call = lambda: K.gemm(M, N, Kd, a, _lib.A_ROWMAJOR, Kd, w, _lib.B_NK, Kd, c, N)  # noqa: E731
            bm = _lib.B_NK
        else:
            w = rnd(Kd, N)
            call = lambda: K.gemm(M, N, Kd, a, _lib.A_ROWMAJOR, Kd, w, _lib.B_KN, N, c, N)  # noqa: E731
            bm = _lib.B_KN
        d = K.GemmDesc()
        d.m, d.n, d.k, d.a_mode, d.b_mode = M, N, Kd, _lib.A_ROWMAJOR, bm
        row = []
        for s in (1, 2, 4):
            K.TUNED = {K.gemm_key(d): s}
            us = timeit(call)
            row.append(f"{s}:{us:6.1f}")
        best = min(float(r.split(":")[1]) for r in row)
        print(f"{mode} M={M:5d} N={N:5d} K={Kd:5d} best {2 * M * N * Kd / best / 1e6:6.1f} TF  " + " ".join(row),
              flush=True)


if __name__ == "__main__":
    main()
