"""Fixed GEMM launches for PMC counter passes (rocprofv3 --pmc ... -- python scripts/gemm_pmc_probe.py): the step's
largest conv forward (variant 2) and conv weight gradient (variants 1 and 4, 6 splits), 10 launches each."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "stablediffusion-pytorch_amd"))
import torch  # noqa: E402

from sdmi import kernels as K  # noqa: E402


def main():
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    rnd = lambda *s: (torch.rand(*s, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)  # noqa: E731
    B, H, cin, cout = 32, 32, 384, 384
    x, dy = rnd(B * H * H, cin), rnd(B * H * H, cout)
    wpk = rnd(cout, 9 * cin)
    out = torch.empty(B * H * H, cout, device=dev, dtype=torch.bfloat16)
    dw = torch.empty(cout, cin, 3, 3, device=dev)
    bg = torch.empty(cout, device=dev)
    gs = torch.empty(B, cout, device=dev, dtype=torch.bfloat16)
    fwd = lambda: K.conv_fwd(x, B, H, H, cin, cin, wpk, cout, 3, 3, 1, 1, out, cout)  # noqa: E731
    wg = lambda: K.conv_wgrad(dy, cout, x, B, H, H, cin, cin, cout, 3, 3, 1, 1, dw, H, H, bias_grad=bg,  # noqa: E731
                              group_sums=gs)
    for fn, cfgs in ((fwd, ([1, 2],)), (wg, ([6, 1], [6, 4]))):
        K.TUNED = {}
        K.GEMM_CAPTURE = []
        fn()
        key = K.gemm_key(K.GEMM_CAPTURE[0])
        K.GEMM_CAPTURE = None
        for c in cfgs:
            K.TUNED = {key: c}
            for _ in range(10):
                fn()
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
