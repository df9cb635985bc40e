"""GroupNorm backward batch-tail check over batch sizes (debug helper)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "stablediffusion-pytorch_amd"))
import torch
import torch.nn.functional as F
from sdmi import kernels as k

for (B, H, C) in [(32, 2, 512), (128, 2, 512), (256, 2, 512), (512, 2, 512), (1024, 2, 512), (1024, 4, 512), (64, 2, 512)]:
    G = 32
    torch.manual_seed(0)
    P = H * H
    x = (torch.randn(B, P, C, device="cuda") * 2 + 0.5).bfloat16()
    gamma = torch.randn(C, device="cuda") * 0.1 + 1
    beta = torch.randn(C, device="cuda") * 0.1
    dy = torch.randn(B, P, C, device="cuda").bfloat16()
    dev = os.environ.get("REF_DEV", "cpu")  # reference device: aten's CPU kernels (double) by default
    xr = x.double().permute(0, 2, 1).to(dev).clone().requires_grad_(True)
    gr = gamma.double().to(dev).clone().requires_grad_(True)
    br = beta.double().to(dev).clone().requires_grad_(True)
    F.silu(F.group_norm(xr, G, gr, br, eps=1e-5)).backward(dy.double().permute(0, 2, 1).to(dev))
    xg, gg, bg = (t.grad.float().cuda() for t in (xr, gr, br))
    x2 = x.view(B * P, C)
    tab = k.gn_stats(x2, B, P, C, G, gamma, beta)
    dx = torch.empty_like(x2)
    dg = torch.empty(C, device="cuda")
    db = torch.empty(C, device="cuda")
    k.gn_bwd(x2, dy.view(B * P, C), dx, tab, gamma, B, P, C, G, True, dg, db)
    torch.cuda.synchronize()
    e = lambda a, b: ((a - b).abs().max() / b.abs().max()).item()
    bad = ((dg - gg).abs() > 0.02 * gg.abs().max()).nonzero().flatten()
    print(dev, B, H, C, "dx", round(e(dx.view(B, P, C).permute(0, 2, 1).float(), xg), 4), "dg", round(e(dg, gg), 4),
          "db", round(e(db, bg), 4), "bad ch", bad[:12].tolist(), len(bad), flush=True)
