import os, sys
REPO = os.getcwd()
sys.path[:0] = [os.path.join(REPO, "stablediffusion-pytorch_amd"), REPO]
import torch
from sdmi import kernels as k
class AllSplit(dict):
    def __init__(s, n): super().__init__(); s.n = n
    def get(s, key, d=0): return s.n
bf = lambda t: t.to(torch.bfloat16)
for (B, H, C, prod, silu) in [(4, 32, 384, "conv", True), (4, 16, 512, "linear", False), (32, 4, 512, "conv", True)]:
    for splits in (1, 4):
        k.TUNED = AllSplit(splits)
        torch.manual_seed(1)
        P, G = H * H, 32
        M = B * P
        x = bf(torch.randn(M, C, device="cuda") * 2 + 0.5)
        gamma = torch.randn(C, device="cuda") * 0.1 + 1
        beta = torch.randn(C, device="cuda") * 0.1
        y = torch.empty_like(x)
        tab = k.gn_fwd(x, B, P, C, G, gamma, beta, silu, y)
        if prod == "conv":
            cu = 256
            g_up = bf(torch.randn(M, cu, device="cuda"))
            wd = bf(torch.randn(C, 9 * cu, device="cuda") * 0.02)
            run = lambda out, gn: k.conv_fwd(g_up, B, H, H, cu, cu, wd, C, 3, 3, 1, 1, out, C, gn=gn)
        else:
            g_up = bf(torch.randn(M, 3 * C, device="cuda"))
            w = bf(torch.randn(3 * C, C, device="cuda") * 0.05)
            run = lambda out, gn: k.linear_dgrad(g_up, w, out, gn=gn)
        dy_ref = torch.empty(M, C, dtype=torch.bfloat16, device="cuda")
        run(dy_ref, None)
        dy = torch.empty_like(dy_ref)
        req = k.gn_request_fwd(P, C) if False else k.gn_request(x, tab, P, C, silu)
        var = __import__("ctypes").c_int(0); tn = __import__("ctypes").c_int(0)
        run(dy, req)
        torch.cuda.synchronize()
        diff = (dy.float() - dy_ref.float()).abs()
        bad = diff > 0
        print(f"B={B} H={H} C={C} {prod} split={splits}: rb={req['rb']} mismatches {int(bad.sum())}/{bad.numel()} max {diff.max().item():.3g}", flush=True)
        if bad.any():
            r, c = bad.nonzero(as_tuple=True)
            print("  rows%128", sorted(set((r % 128).tolist()))[:20], " cols%192", sorted(set((c % 192).tolist()))[:30], flush=True)
            print("  rows", r[:10].tolist(), "cols", c[:10].tolist(), flush=True)
            print("  ref", dy_ref[r[:5], c[:5]].tolist(), "got", dy[r[:5], c[:5]].tolist(), flush=True)
        add = bf(torch.randn(M, C, device="cuda"))
        dx_ref, dx = torch.empty_like(x), torch.empty_like(x)
        dg_ref, db_ref, dg, db = (torch.empty(C, device="cuda") for _ in range(4))
        k.gn_bwd(x, dy_ref, dx_ref, tab, gamma, B, P, C, G, silu, dg_ref, db_ref, addend=add)
        k.gn_bwd(x, dy_ref, dx, tab, gamma, B, P, C, G, silu, dg, db, addend=add, gn=req)
        torch.cuda.synchronize()
        rel = lambda a, b: ((a.float() - b.float()).abs().max() / b.float().abs().max()).item()
        print(f"  dx rel {rel(dx, dx_ref):.3g} dg rel {rel(dg, dg_ref):.3g} db rel {rel(db, db_ref):.3g}", flush=True)
