"""Isolated GroupNorm(+SiLU) forward / backward timings at the cond-UNet step shapes (B=32): achieved HBM rate of
the algorithmic bytes (fwd: read x + write y = 4 B/elem; bwd: read x, dy + write dx = 6 B/elem)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "stablediffusion-pytorch_amd"))
import torch
from sdmi import kernels as k


def timeit(fn, iters=50):
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


B, G = 32, 32
for (H, C) in [(32, 256), (32, 384), (32, 768), (32, 128), (16, 512), (16, 384), (16, 1024), (8, 768), (8, 512), (4, 768)]:
    P = H * H
    x = torch.randn(B * P, C, device="cuda").bfloat16()
    dy = torch.randn(B * P, C, device="cuda").bfloat16()
    gamma = torch.ones(C, device="cuda")
    beta = torch.zeros(C, device="cuda")
    y = torch.empty_like(x)
    dx = torch.empty_like(x)
    dg = torch.empty(C, device="cuda")
    db = torch.empty(C, device="cuda")
    tab = k.gn_fwd(x, B, P, C, G, gamma, beta, True, y)
    tf = timeit(lambda: k.gn_fwd(x, B, P, C, G, gamma, beta, True, y))
    tb = timeit(lambda: k.gn_bwd(x, dy, dx, tab, gamma, B, P, C, G, True, dg, db))
    tn = timeit(lambda: k.gn_bwd(x, dy, dx, tab, gamma, B, P, C, G, True, None, None))  # no dgamma / dbeta tail
    n = B * P * C
    print(f"{H:3d}^2 C={C:5d}: fwd {tf:7.1f} us {4 * n / tf / 1e6:6.2f} TB/s | bwd {tb:7.1f} us {6 * n / tb / 1e6:6.2f} TB/s"
          f" | bwd w/o param grads {tn:7.1f} us", flush=True)
