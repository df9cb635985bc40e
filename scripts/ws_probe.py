"""Isolated timing of the warp-specialised persistent GEMM (variants 12 / 13) against the tuned table's mainloops on the
short-K row-major shapes of the cond-UNet / DiT steps (bias + residual epilogue, bf16 out; HIP events, median of 5 x 20
back-to-back launches). Usage: python scripts/ws_probe.py"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "stablediffusion-pytorch_amd"), REPO]
import torch  # noqa: E402

SHAPES = [(8192, 1152, 288), (8192, 864, 288), (8192, 288, 1152), (8192, 288, 288), (32768, 384, 384),
          (32768, 1152, 384), (32768, 384, 1152), (8192, 512, 512), (2048, 768, 768), (32768, 128, 128)]
VARIANTS = [int(v) for v in os.environ.get("WS_VARIANTS", "2,9,10,12,13").split(",")]


def main():
    from sdmi import kernels as K, _lib as L
    dev = torch.device("cuda", 0)
    for M, N, Kd in SHAPES:
        a = torch.randn(M, Kd, device=dev).to(torch.bfloat16)
        w = (torch.randn(N, Kd, device=dev) * 0.05).to(torch.bfloat16)
        bias = torch.randn(N, device=dev)
        res = torch.randn(M, N, device=dev).to(torch.bfloat16)
        c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        row = []
        for v in VARIANTS:
            K.TUNED = {"__all__": [1, v]}
            K.gemm_key = lambda d: "__all__"
            run = lambda: K.gemm(M, N, Kd, a, L.A_ROWMAJOR, Kd, w, L.B_NK, Kd, c, N, bias=bias, resid=res, ldr=N)  # noqa
            for _ in range(3):
                run()
            ts = []
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(20):
                    run()
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3 / 20)
            row.append(sorted(ts)[2])
        fl = 2.0 * M * N * Kd
        best = min(range(len(VARIANTS)), key=lambda i: row[i])
        print(f"M={M:6d} N={N:5d} K={Kd:5d}  " + "  ".join(f"v{v}:{t:6.1f}" for v, t in zip(VARIANTS, row)) +
              f"   best v{VARIANTS[best]} {fl / row[best] / 1e6:.0f} TF", flush=True)


if __name__ == "__main__":
    main()
