"""Where in the cond-UNet backward the flat gradient buffer becomes final (the DP all-reduce watermarks of
sdmi.trainer): for each backward tape position, the flat prefix (MB) that is final and the device time elapsed.
Shows how much of the 474 MB gradient is only final at the very end (the all-reduce tail no overlap can hide).
Usage (GPU): python scripts/bucket_marks.py"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "stablediffusion-pytorch_amd"))
import torch  # noqa: E402


def main():
    from tests.golden.configs import full_cond_config
    from sdmi.trainer import DDPMTrainer
    import models.unet_cond_base as mc
    import bench
    cfg = full_cond_config()
    dev = torch.device("cuda", 0)
    torch.manual_seed(1111)
    tr = DDPMTrainer(cfg, mc.Unet(4, cfg).state_dict(), dev)
    x0, text, empty, mask = bench.synthetic_batch(32, dev, 1111)
    noise = torch.randn_like(x0)
    t = torch.randint(0, 1000, (32,), device=dev)
    keep = torch.ones(32, device=dev)
    for _ in range(2):
        tr.step(x0, noise, t, text, mask, mask_keep=keep)
    torch.cuda.synchronize()
    eng = tr.engine
    pred, ctx = eng.forward(tr._xt if hasattr(tr, "_xt") else x0, t, text, mask, mask_keep=keep)
    tape = ctx["tape"] if isinstance(ctx, dict) else ctx
    marks = tr._watermarks(tape)
    total = tr.store.numel * 4
    rows = []
    for k in range(len(tape) - 1, -1, -1):
        upto = 0
        for end, run in marks:
            if run >= k:
                upto = end
            else:
                break
        rows.append((len(tape) - 1 - k, tape[k][1].get("label"), upto * 4 / 1e6))
    last = 0.0
    for i, lab, mb in rows:
        if mb != last:
            print(f"after backward entry {i:4d}/{len(tape)} ({lab}): final prefix {mb:8.1f} MB of {total / 1e6:.1f}")
            last = mb
    print(f"final only at the end: {(total / 1e6) - max((r[2] for r in rows[:-1]), default=0):.1f} MB")


if __name__ == "__main__":
    main()
