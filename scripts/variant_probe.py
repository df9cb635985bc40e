"""Mainloop-variant probe on the step's characteristic GEMM shapes: for each shape, the best isolated time per
mainloop variant (1 register-staged, 2 / 3 LDS-DMA 128-row tiles, 4 LDS-DMA large 8-wave tiles) over the split
counts, with the bias / group-sum reductions the step requests on weight gradients.
Usage: python scripts/variant_probe.py [variants, default 1,2,4]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "stablediffusion-pytorch_amd"))
import torch  # noqa: E402

from sdmi import kernels as K, _lib  # noqa: E402

SPLITS = (1, 2, 3, 4, 6, 8, 12, 16, 24, 32)


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
    variants = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "1,2,4").split(",")]
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    rnd = lambda *s: (torch.rand(*s, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)  # noqa: E731
    cases = []
    B = 32
    for (cout, cin, H) in ((384, 384, 32), (512, 512, 16), (128, 128, 32), (768, 768, 8)):
        x, dy = rnd(B * H * H, cin), rnd(B * H * H, cout)
        dw = torch.empty(cout, cin, 3, 3, device=dev)
        bg = torch.empty(cout, device=dev)
        gs = torch.empty(B, cout, device=dev, dtype=torch.bfloat16)
        cases.append((f"conv wgrad {cout}x{9 * cin}x{B * H * H}", 2.0 * cout * 9 * cin * B * H * H,
                      lambda x=x, dy=dy, dw=dw, bg=bg, gs=gs, cout=cout, cin=cin, H=H: K.conv_wgrad(
                          dy, cout, x, B, H, H, cin, cin, cout, 3, 3, 1, 1, dw, H, H, bias_grad=bg, group_sums=gs)))
        wpk = rnd(cout, 9 * cin)
        out = torch.empty(B * H * H, cout, device=dev, dtype=torch.bfloat16)
        cases.append((f"conv fwd {B * H * H}x{cout}x{9 * cin}", 2.0 * cout * 9 * cin * B * H * H,
                      lambda x=x, wpk=wpk, out=out, cout=cout, cin=cin, H=H: K.conv_fwd(
                          x, B, H, H, cin, cin, wpk, cout, 3, 3, 1, 1, out, cout)))
    for (M, N, Kd) in ((384, 384, 32768), (1152, 384, 32768), (512, 512, 8192)):
        a, b = rnd(Kd, M), rnd(Kd, N)
        c = torch.empty(M, N, device=dev)
        bg = torch.empty(M, device=dev)
        cases.append((f"linear wgrad {M}x{N}x{Kd}", 2.0 * M * N * Kd,
                      lambda a=a, b=b, c=c, bg=bg, M=M, N=N, Kd=Kd: K.linear_wgrad(
                          a[:, :M].view(Kd, M), b, c, bias_grad=bg)))
    for name, fl, fn in cases:
        K.TUNED = {}
        K.GEMM_CAPTURE = []
        fn()
        d = K.GEMM_CAPTURE[0]
        K.GEMM_CAPTURE = None
        key = K.gemm_key(d)
        row = []
        for v in variants:
            best = (1e9, 0)
            for s in SPLITS:
                K.TUNED = {key: [s, v]}
                us = timeit(fn)
                best = min(best, (us, s))
            row.append(f"v{v}: {best[0]:7.1f} us s{best[1]:<2d} {fl / best[0] / 1e6:6.1f} TF")
        print(f"{name:34s} " + " | ".join(row), flush=True)


if __name__ == "__main__":
    main()
