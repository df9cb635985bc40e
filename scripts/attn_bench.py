"""Attention kernel timing at the cond-UNet / DiT shapes (B=32): forward and backward, microseconds."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "stablediffusion-pytorch_amd"))
import torch  # noqa: E402

from sdmi import kernels as K  # noqa: E402


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
    bf = torch.bfloat16
    shapes = ((32, 16, 1024, 1024, 8), (32, 16, 1024, 1024, 16), (32, 16, 1024, 1024, 24), (32, 16, 1024, 77, 8), (32, 16, 1024, 77, 16), (32, 16, 1024, 77, 24),
              (32, 16, 256, 256, 24), (32, 16, 256, 256, 32), (32, 16, 64, 64, 32), (32, 16, 64, 64, 48),
              (32, 16, 16, 16, 48), (32, 9, 256, 256, 32))
    if len(sys.argv) > 1:  # one shape index (for per-kernel rocprof runs)
        shapes = (shapes[int(sys.argv[1])],)
    for (B, H, N, S, d) in shapes:
        C = H * d
        amp = float(os.environ.get("ATTN_AMP", "1"))  # input scale (score magnitude)
        q = (torch.randn(B * N, C, device=dev) * amp).to(bf)
        k = (torch.randn(B * S, C, device=dev) * amp).to(bf)
        v = torch.randn(B * S, C, device=dev).to(bf)
        o = torch.empty(B * N, C, device=dev, dtype=bf)
        lse = [None]

        def fwd():
            lse[0] = K.attn_fwd(q, k, v, o, B, H, N, S, d)
        tf = timeit(fwd)
        do = torch.randn(B * N, C, device=dev).to(bf)
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        tb = timeit(lambda: K.attn_bwd(q, k, v, o, do, lse[0], dq, dk, dv, B, H, N, S, d))
        fl = 4.0 * B * H * N * S * d
        print(f"B={B} H={H:2d} N={N:4d} S={S:4d} d={d:2d}: fwd {tf:7.1f} us ({fl / tf / 1e6:6.1f} TF)  "
              f"bwd {tb:7.1f} us ({2.5 * fl / tb / 1e6:6.1f} TF)", flush=True)


if __name__ == "__main__":
    main()
