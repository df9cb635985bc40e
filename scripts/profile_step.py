"""Per-launch timing of one cond-UNet training step (HIP events around every sdmi launch group).
Usage: python scripts/profile_step.py [--batch 32] [--top 40]"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "stablediffusion-pytorch_amd"), REPO]
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--dump", default="", help="write every launch (in issue order) to this file")
    args = ap.parse_args()
    from sdmi.trainer import DDPMTrainer
    from sdmi import kernels as K
    import models.unet_cond_base as mc
    dev = torch.device("cuda", 0)
    cfg = bench.cond_config()
    torch.manual_seed(0)
    tr = DDPMTrainer(cfg, mc.Unet(4, cfg).state_dict(), dev)
    B = args.batch
    x0, text, empty, mask = bench.synthetic_batch(B, dev, 1)

    def step():
        noise = torch.randn_like(x0)
        t = torch.randint(0, 1000, (B,), device=dev)
        tr.step(x0, noise, t, text, mask, mask_keep=torch.ones(B, device=dev))

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    K.PROFILE = []
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    step()
    e1.record()
    torch.cuda.synchronize()
    prof, K.PROFILE = K.PROFILE, None
    rows = [(tag, fl, a.elapsed_time(b), info) for tag, fl, a, b, info in prof]
    total = e0.elapsed_time(e1)
    print(f"step wall (events) {total:.3f} ms; profiled launches {sum(r[2] for r in rows):.3f} ms")
    agg = {}
    for tag, fl, ms, info in rows:
        a = agg.setdefault(tag, [0, 0.0, 0.0])
        a[0] += 1
        a[1] += ms
        a[2] += fl
    for tag, (n, ms, fl) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        tf = fl / (ms * 1e-3) / 1e12 if fl else 0
        print(f"{tag:14s} {n:5d} launches {ms:8.3f} ms  {tf:7.1f} TFLOP/s")
    if args.dump:
        with open(args.dump, "w") as f:
            for tag, fl, ms, info in rows:
                f.write(f"{ms * 1000:9.1f} us  {tag:12s} {info}\n")
    print("--- top launches ---")
    for tag, fl, ms, info in sorted(rows, key=lambda r: -r[2])[:args.top]:
        tf = fl / (ms * 1e-3) / 1e12 if fl else 0
        print(f"{ms * 1000:8.1f} us {tf:7.1f} TF  {tag:12s} {info}")


if __name__ == "__main__":
    main()
