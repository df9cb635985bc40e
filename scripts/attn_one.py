"""One attention shape, forward (and optionally backward), a few launches: a short target for rocprofv3 --pmc passes.
Usage: python scripts/attn_one.py B H N S d [fwd|bwd]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "stablediffusion-pytorch_amd"))
import torch  # noqa: E402

from sdmi import kernels as K  # noqa: E402


def main():
    B, H, N, S, d = (int(x) for x in sys.argv[1:6])
    what = sys.argv[6] if len(sys.argv) > 6 else "fwd"
    dev, bf = "cuda", torch.bfloat16
    C = H * d
    q = torch.randn(B * N, C, device=dev).to(bf)
    k = torch.randn(B * S, C, device=dev).to(bf)
    v = torch.randn(B * S, C, device=dev).to(bf)
    o = torch.empty(B * N, C, device=dev, dtype=bf)
    lse = K.attn_fwd(q, k, v, o, B, H, N, S, d)
    do = torch.randn(B * N, C, device=dev).to(bf)
    dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    for _ in range(5):
        if what == "fwd":
            K.attn_fwd(q, k, v, o, B, H, N, S, d)
        else:
            K.attn_bwd(q, k, v, o, do, lse, dq, dk, dv, B, H, N, S, d)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
