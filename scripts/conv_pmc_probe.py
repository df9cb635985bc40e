"""The 32^2 3x3 conv of the cond-UNet (B = 32, 384 -> 384 channels) as forward and as weight gradient, one case per
run (argv[1]: fwd | wg<split>v<variant>), 5 launches each after 2 warm-ups, for per-kernel rocprofv3 SQ counters
(scripts/gpu_conv_pmc.sh): where the weight-gradient mainloop loses against the forward at the same FLOPs."""
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "stablediffusion-pytorch_amd")]
import torch  # noqa: E402


def main():
    from sdmi import kernels as K
    case = sys.argv[1]
    B, H, C = 32, 32, 384
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(B * H * H, C, device="cuda", generator=g).to(torch.bfloat16)
    w = torch.randn(C, 9 * C, device="cuda", generator=g).to(torch.bfloat16)
    y = torch.randn(B * H * H, C, device="cuda", generator=g).to(torch.bfloat16)
    dw = torch.empty(C, 9 * C, device="cuda")
    if case == "fwd":
        fn = lambda: K.conv_fwd(x, B, H, H, C, C, w, C, 3, 3, 1, 1, y, C)  # noqa: E731
    else:
        sp, v = case[2:].split("v")
        K.TUNED = {"__all__": [int(sp), int(v)]}
        K.gemm_key = lambda d: "__all__"
        fn = lambda: K.conv_wgrad(y, C, x, B, H, H, C, C, C, 3, 3, 1, 1, dw, H, H)  # noqa: E731
    for _ in range(2):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(5):
        fn()
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) / 5 * 1e3
    print(f"{case}: {us:.1f} us/launch, {2 * B * H * H * C * 9 * C / us / 1e6:.0f} TF", flush=True)


if __name__ == "__main__":
    main()
