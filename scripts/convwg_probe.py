"""Conv weight-gradient GEMM probe (col-major dY^T x implicit im2col(x)): time per split count for the step's
3x3 shapes. Run once per SDMI_GEMM_VARIANT. Usage: SDMI_GEMM_VARIANT=0 python scripts/convwg_probe.py"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "stablediffusion-pytorch_amd"))
import torch  # noqa: E402

from sdmi import kernels as K, _lib  # noqa: E402

SHAPES = ((32, 32, 384, 384), (32, 32, 128, 128), (32, 32, 384, 128), (32, 16, 256, 256), (32, 16, 512, 512),
          (32, 8, 768, 768), (32, 8, 512, 512))


def timeit(fn, iters=10):
    for _ in range(2):
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
    splits = [int(x) for x in os.environ.get("SPLITS", "1,2,4,8,16,32").split(",")]
    for (B, H, cin, cout) in SHAPES:
        x, dy = rnd(B * H * H, cin), rnd(B * H * H, cout)
        dw = torch.empty(cout, cin, 3, 3, device=dev)
        row = []
        for s in splits:
            K.TUNED = {"-": 0}  # non-empty: the launch looks its key up
            # key of this launch: record it through the tuned-table lookup
            keys = []
            orig = K.gemm_key
            K.gemm_key = lambda d: keys.append(orig(d)) or orig(d)  # noqa: E731
            K.conv_wgrad(dy, cout, x, B, H, H, cin, cin, cout, 3, 3, 1, 1, dw, H, H)
            K.gemm_key = orig
            K.TUNED = {keys[0]: s}
            us = timeit(lambda: K.conv_wgrad(dy, cout, x, B, H, H, cin, cin, cout, 3, 3, 1, 1, dw, H, H))
            row.append(f"{s}:{us:6.1f}")
        fl = 2.0 * B * H * H * cin * cout * 9
        best = min(float(r.split(":")[1]) for r in row)
        print(f"B={B} {H}x{H} {cin}->{cout} best {fl / best / 1e6:6.1f} TF  " + " ".join(row), flush=True)


if __name__ == "__main__":
    main()
