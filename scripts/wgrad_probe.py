"""Weight-gradient GEMM probe (col-major A = activations^T / dY^T, long K = pixels): time per split count for the
step's shapes. Run once per SDMI_GEMM_VARIANT. Usage: SDMI_GEMM_VARIANT=0 python scripts/wgrad_probe.py"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "stablediffusion-pytorch_amd"))
import torch  # noqa: E402

from sdmi import kernels as K, _lib  # noqa: E402

SHAPES = ((1152, 384, 32768), (384, 384, 32768), (128, 128, 32768), (384, 128, 32768), (128, 512, 32768),
          (1536, 512, 8192), (512, 512, 8192), (2304, 768, 2048), (768, 768, 2048))


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
    splits = [int(x) for x in os.environ.get("SPLITS", "1,2,4,8,16,32,64,128").split(",")]
    for (M, N, Kd) in SHAPES:
        a, b = rnd(Kd, M), rnd(Kd, N)
        c = torch.empty(M, N, device=dev, dtype=torch.float32)
        row = []
        for s in splits:
            K.TUNED = {"__force__": 1}
            d = K.GemmDesc() if hasattr(K, "GemmDesc") else _lib.GemmDesc()
            d.m, d.n, d.k, d.a_mode, d.b_mode = M, N, Kd, _lib.A_COLMAJOR, _lib.B_KN
            key = K.gemm_key(d)
            K.TUNED = {key: s}
            us = timeit(lambda: K.gemm(M, N, Kd, a, _lib.A_COLMAJOR, M, b, _lib.B_KN, N, c, N))
            row.append(f"{s}:{us:6.1f}")
        print(f"M={M:5d} N={N:4d} K={Kd:5d} best {2 * M * N * Kd / min(float(r.split(':')[1]) for r in row) / 1e6:6.1f} TF  "
              + " ".join(row), flush=True)


if __name__ == "__main__":
    main()
