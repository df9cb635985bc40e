"""Per-call device time of the linear data-gradient GEMMs of one cond-UNet step (single stream), from the
transposed weight (B_NK, SDMI_DGRAD_T=1) against the forward weight (B_KN, =0). Usage: python scripts/dgrad_compare.py"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "stablediffusion-pytorch_amd"), REPO]
os.environ["SDMI_WG_STREAM"] = "0"
import torch  # noqa: E402

import bench  # noqa: E402


def run(flag):
    os.environ["SDMI_DGRAD_T"] = flag
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
    out = []
    for rep in range(5):
        K.PROFILE = []
        tr.step(x0, noise, t, text, mask, mask_keep=keep)
        torch.cuda.synchronize()
        prof, K.PROFILE = K.PROFILE, None
        calls = [(tag, info, a.elapsed_time(b)) for tag, fl, a, b, info in prof
                 if info.startswith("[bwd]") and tag in ("gemm_a0b1", "gemm_a0b0")]
        if not out:
            out = [[tag, info, [ms]] for tag, info, ms in calls]
        else:
            for o, (_, _, ms) in zip(out, calls):
                o[2].append(ms)
    return [(tag, info, sorted(ms)[len(ms) // 2]) for tag, info, ms in out]


def main():
    r = {f: run(f) for f in ("0", "1")}
    t0 = t1 = 0.0
    for (ta, ia, ma), (tb, ib, mb) in zip(r["0"], r["1"]):
        t0 += ma
        t1 += mb
        print(f"{ma * 1e3:7.1f} us {ta} -> {mb * 1e3:7.1f} us {tb}   {ia[:70]} | {ib[:70]}")
    print(f"total {t0:.3f} -> {t1:.3f} ms")


if __name__ == "__main__":
    main()
