"""Host issue time of one plan-replayed cond-UNet training step, and a device-true kernel timeline for profiling.

1. host: median wall time of ONE replay() call issued onto an idle GPU (no sync inside), i.e. the C++ launch loop
   plus the Python callouts, against the synced step time;
2. timeline: the main stream is parked behind a long spin kernel while TIMELINE_STEPS steps are enqueued, so under
   rocprofv3 --kernel-trace the recorded steps run back to back at device speed (the tracer's per-launch host
   cost no longer shows up as gaps). scripts/critical_path.py then reads the trace.
Usage: python scripts/device_step.py [--workload cond-unet|dit|uncond-unet] [--timeline-steps 2]"""
import argparse
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "stablediffusion-pytorch_amd"), REPO]
import torch  # noqa: E402

import bench  # noqa: E402


def make(workload, dev):
    from sdmi.trainer import DDPMTrainer
    from sdmi.graph import CapturedTrainStep
    torch.manual_seed(1111)
    B = 32
    x0, text, empty, mask = bench.synthetic_batch(B, dev, 1111)
    gen = torch.Generator(device=dev).manual_seed(1111)
    if workload == "dit":
        from models.transformer import DIT
        cfg = bench.dit_config()
        init = DIT(4, cfg).state_dict()
        for v in init.values():
            if v.abs().max() == 0:
                v.normal_(0.0, 0.02)
        tr = DDPMTrainer(cfg, init, dev, base="dit", lr=1e-4, ema_decay=None)
        return CapturedTrainStep(tr, x0, None, empty, mask, B, generator=gen, drop_p=0.9)
    if workload == "uncond-unet":
        import models.unet_base as mu
        cfg = bench.uncond_config()
        tr = DDPMTrainer(cfg, mu.Unet(4, cfg).state_dict(), dev, base="uncond", lr=5e-6, ema_decay=None,
                         max_grad_norm=float("inf"), sched=(1000, 0.0015, 0.0195))
        return CapturedTrainStep(tr, x0, None, empty, None, B, generator=gen)
    import models.unet_cond_base as mc
    cfg = bench.cond_config()
    tr = DDPMTrainer(cfg, mc.Unet(4, cfg).state_dict(), dev)
    return CapturedTrainStep(tr, x0, text, empty, mask, B, generator=gen)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="cond-unet")
    ap.add_argument("--timeline-steps", type=int, default=2)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from sdmi import streams
    streams.reserve(dev)  # as bench.py: the engines' streams on queues of their own
    cap = make(a.workload, dev)
    for _ in range(3):
        cap.step()
    torch.cuda.synchronize()
    n, k, c = cap.plan.info()
    host, wall = [], []
    for _ in range(7):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        cap.step()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        host.append(t1 - t0)
        wall.append(t2 - t0)
    print(f"plan: {n} ops, {k} kernel launches, {c} callouts; host issue {1e3 * statistics.median(host):.2f} ms/step, "
          f"issue+drain {1e3 * statistics.median(wall):.2f} ms/step", flush=True)
    if a.timeline_steps > 0:
        torch.cuda.synchronize()
        torch.cuda._sleep(int(os.environ.get("SPIN_CYCLES", "400000000")))  # park the main stream
        t0 = time.perf_counter()
        for _ in range(a.timeline_steps):
            cap.step()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"timeline: {a.timeline_steps} steps enqueued in {1e3 * (t1 - t0):.1f} ms behind the spin, "
              f"drained at {1e3 * (t2 - t0):.1f} ms", flush=True)


if __name__ == "__main__":
    main()
