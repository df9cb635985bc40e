"""Per-phase device time of one cond-UNet step (single stream, no overlap): forward, backward data-gradient
chain and weight-gradient work, by kernel family. Usage: python scripts/phase_profile.py"""
import collections
import os
import re
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "stablediffusion-pytorch_amd"), REPO]
os.environ["SDMI_WG_STREAM"] = "0"
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    from sdmi.trainer import DDPMTrainer
    from sdmi import kernels as K
    import models.unet_cond_base as mc
    dev = torch.device("cuda", 0)
    cfg = bench.cond_config()
    torch.manual_seed(0)
    tr = DDPMTrainer(cfg, mc.Unet(4, cfg).state_dict(), dev)
    B = 32
    x0, text, empty, mask = bench.synthetic_batch(B, dev, 1)
    noise = torch.randn_like(x0)
    t = torch.randint(0, 1000, (B,), device=dev)
    keep = torch.ones(B, device=dev)
    for _ in range(3):
        tr.step(x0, noise, t, text, mask, mask_keep=keep)
    torch.cuda.synchronize()
    K.PROFILE = []
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    tr.step(x0, noise, t, text, mask, mask_keep=keep)
    e1.record()
    torch.cuda.synchronize()
    prof, K.PROFILE = K.PROFILE, None
    total = e0.elapsed_time(e1)
    agg = collections.defaultdict(float)
    ph = collections.defaultdict(float)
    for tag, fl, a, b, info in prof:
        m = re.match(r"\[(\w+)\]", info)
        phase = m.group(1) if m else "other"
        ms = a.elapsed_time(b)
        agg[(phase, tag)] += ms
        ph[phase] += ms
    print(f"step {total:.3f} ms (single stream); profiled {sum(ph.values()):.3f} ms")
    for p, ms in sorted(ph.items(), key=lambda kv: -kv[1]):
        print(f"  {p:6s} {ms:7.3f} ms")
    for (p, tag), ms in sorted(agg.items(), key=lambda kv: -kv[1]):
        print(f"  {p:6s} {tag:12s} {ms:7.3f} ms")


if __name__ == "__main__":
    main()
