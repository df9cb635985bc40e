"""Where the weight-gradient GEMMs' time goes: each of the step's conv / linear weight-gradient shapes timed with
(a) the step's output layout (torch (co, ci, kh, kw): column-permuted scalar epilogue) and bias reductions,
(b) the GEMM-natural layout (co, kh, kw, ci) through the 16-B vector epilogue, no bias, for mainloop variants 0 / 2
and a sweep of split counts. Run under rocprofv3 --kernel-trace --stats to split GEMM and reducer time.
Usage: python scripts/wg_anatomy.py"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "stablediffusion-pytorch_amd"))
import torch  # noqa: E402

from sdmi import kernels as K  # noqa: E402

CONV = ((32, 4, 512, 512), (32, 8, 768, 768), (32, 16, 512, 512), (32, 32, 384, 384))
LIN = ((32768, 384, 384), (8192, 512, 512), (512, 512, 512), (2048, 768, 768), (32768, 128, 128))


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


def with_hint(fn, s, v):
    keys = []
    orig = K.gemm_key
    K.TUNED = {"-": 0}
    K.gemm_key = lambda d: keys.append(orig(d)) or orig(d)  # noqa: E731
    fn()
    K.gemm_key = orig
    K.TUNED = {keys[0]: [s, v]}
    return timeit(fn)


def main():
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    rnd = lambda *s: (torch.rand(*s, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)  # noqa: E731
    splits = [int(x) for x in os.environ.get("SPLITS", "1,2,4,8,16").split(",")]
    for (B, H, cin, cout) in CONV:
        x, dy = rnd(B * H * H, cin), rnd(B * H * H, cout)
        dw = torch.empty(cout, cin, 3, 3, device=dev)
        bg, bg2 = torch.empty(cout, device=dev), torch.empty(cout, device=dev)
        fl = 2.0 * B * H * H * cin * cout * 9
        forms = {
            "torch+bias": lambda: K.conv_wgrad(dy, cout, x, B, H, H, cin, cin, cout, 3, 3, 1, 1, dw, H, H,
                                               bias_grad=bg, bias_grad2=bg2),
            "torch": lambda: K.conv_wgrad(dy, cout, x, B, H, H, cin, cin, cout, 3, 3, 1, 1, dw, H, H),
            "natural": lambda: K.conv_wgrad(dy, cout, x, B, H, H, cin, cin, cout, 3, 3, 1, 1, dw, H, H, perm=False),
        }
        for name, fn in forms.items():
            for v in (1, 2):
                row = []
                for s in splits:
                    us = with_hint(fn, s, v)
                    row.append(f"{s}:{us:6.1f}")
                best = min(float(r.split(":")[1]) for r in row)
                print(f"conv B={B} {H}x{H} {cin}->{cout} {name:10s} v{v} best {fl / best / 1e6:6.1f} TF  "
                      + " ".join(row), flush=True)
    for (M, N, Kd) in LIN:
        dy, x = rnd(M, N), rnd(M, Kd)
        dw = torch.empty(N, Kd, device=dev)
        bg = torch.empty(N, device=dev)
        fl = 2.0 * M * N * Kd
        forms = {"bias": lambda: K.linear_wgrad(dy, x, dw, bias_grad=bg), "plain": lambda: K.linear_wgrad(dy, x, dw)}
        for name, fn in forms.items():
            for v in (1, 2):
                row = []
                for s in splits + [24, 32, 64]:
                    us = with_hint(fn, s, v)
                    row.append(f"{s}:{us:6.1f}")
                best = min(float(r.split(":")[1]) for r in row)
                print(f"lin M={M} {N}x{Kd} {name:6s} v{v} best {fl / best / 1e6:6.1f} TF  " + " ".join(row), flush=True)


if __name__ == "__main__":
    main()
