"""GroupNorm backward at the cond-UNet's B=32 shapes, with (GN_TAIL=1) or without (GN_TAIL=0) the dgamma/dbeta
batch tail; run under `rocprofv3 --kernel-trace --stats` to read device times free of the Python launch cost.
Usage: GN_TAIL=0|1 python scripts/gn_tail_probe.py"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "stablediffusion-pytorch_amd"))
import torch  # noqa: E402

from sdmi import kernels as K  # noqa: E402


def main():
    tail = os.environ.get("GN_TAIL", "1") == "1"
    dev = "cuda"
    torch.manual_seed(0)
    B, G = 32, 32
    for (P, C) in ((16, 768), (16, 512), (64, 768), (64, 512), (256, 512), (256, 768), (1024, 256), (1024, 384)):
        x = torch.randn(B * P, C, device=dev).to(torch.bfloat16)
        dy = torch.randn(B * P, C, device=dev).to(torch.bfloat16)
        dx = torch.empty_like(dy)
        gamma, beta = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev)
        y = torch.empty_like(x)
        tab = K.gn_fwd(x, B, P, C, G, gamma, beta, True, y)
        dg, db = (torch.empty(C, device=dev), torch.empty(C, device=dev)) if tail else (None, None)
        for _ in range(20):
            K.gn_bwd(x, dy, dx, tab, gamma, B, P, C, G, True, dg, db)
        torch.cuda.synchronize()
        print(f"P={P} C={C} done", flush=True)


if __name__ == "__main__":
    main()
