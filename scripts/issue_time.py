"""Host issue cost vs device time of one cond-UNet training step: is the step launch-bound?
Prints the host time to enqueue a step (no sync), the synced step time, and the graph-replay step time."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "stablediffusion-pytorch_amd"), REPO]
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    from sdmi.trainer import DDPMTrainer
    from sdmi.graph import CapturedTrainStep
    import models.unet_cond_base as mc
    dev = torch.device("cuda", 0)
    cfg = bench.cond_config()
    torch.manual_seed(0)
    tr = DDPMTrainer(cfg, mc.Unet(4, cfg).state_dict(), dev)
    B = 32
    x0, text, empty, mask = bench.synthetic_batch(B, dev, 1)
    keep = torch.ones(B, device=dev)

    def step():
        noise = torch.randn_like(x0)
        t = torch.randint(0, 1000, (B,), device=dev)
        tr.step(x0, noise, t, text, mask, mask_keep=keep)

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    # host issue time while the GPU is busy with a long queue
    n = 10
    t0 = time.perf_counter()
    for _ in range(n):
        step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"eager: host issue {1e3 * (t1 - t0) / n:.2f} ms/step, wall {1e3 * (t2 - t0) / n:.2f} ms/step")
    from sdmi.plan import StepPlan
    noise = torch.randn_like(x0)
    t = torch.randint(0, 1000, (B,), device=dev)
    plan = StepPlan(lambda: tr.step(x0, noise, t, text, mask, mask_keep=keep), dev)
    for _ in range(3):
        plan.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        plan.replay()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"native plan: host issue {1e3 * (t1 - t0) / n:.2f} ms/step, wall {1e3 * (t2 - t0) / n:.2f} ms/step")
    # the loops above saturate the HIP queue (the host blocks once ~1 step is in flight): the host cost of ONE step is
    # its enqueue time from an idle GPU (median of 5), well inside the step's device time
    def one(fn):
        ts = []
        for _ in range(5):
            torch.cuda.synchronize()
            a = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - a)
            torch.cuda.synchronize()
        return 1e3 * sorted(ts)[2]
    print(f"single step from idle: eager enqueue {one(step):.2f} ms, native plan enqueue {one(plan.replay):.2f} ms")
    cap = CapturedTrainStep(tr, x0, text, empty, mask, B)
    for _ in range(3):
        cap.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        cap.step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"graph: host issue {1e3 * (t1 - t0) / n:.2f} ms/step, wall {1e3 * (t2 - t0) / n:.2f} ms/step")


if __name__ == "__main__":
    main()
