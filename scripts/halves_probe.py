"""How latency-bound is the cond-UNet forward at B = 32? The forward recorded once as a native plan (sdmi.plan) three
ways and replayed: the whole batch on one stream, two half batches on two streams, four quarter batches on four
streams (the same kernels on fewer rows each; the halves share the weights). If the small levels are bound by kernel
latency rather than throughput, the concurrent sub-batch chains overlap it."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "stablediffusion-pytorch_amd"), REPO]
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    from sdmi.trainer import DDPMTrainer
    from sdmi import plan
    import models.unet_cond_base as mc
    dev = torch.device("cuda", 0)
    cfg = bench.cond_config()
    torch.manual_seed(0)
    tr = DDPMTrainer(cfg, mc.Unet(4, cfg).state_dict(), dev)
    eng = tr.engine
    eng.refresh_weights()
    B = 32
    x0, text, empty, mask = bench.synthetic_batch(B, dev, 1)
    t = torch.randint(0, 1000, (B,), device=dev)
    streams = [torch.cuda.Stream(device=dev) for _ in range(4)]

    def split(n):
        def fn():
            cur = torch.cuda.current_stream(dev)
            ev = torch.cuda.Event()
            plan.record_event(ev, cur)
            ends = []
            for i in range(n):
                s = streams[i]
                plan.wait_event(s, ev)
                sl = slice(i * B // n, (i + 1) * B // n)
                with torch.cuda.stream(s):
                    eng.forward(x0[sl], t[sl], text[sl], mask[sl], need_backward=False)
                e = torch.cuda.Event()
                plan.record_event(e, s)
                ends.append(e)
            for e in ends:
                plan.wait_event(cur, e)
        return fn

    for n in (1, 2, 4):
        fn = split(n)
        fn()
        torch.cuda.synchronize()
        p = plan.StepPlan(fn, dev)
        for _ in range(3):
            p.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            p.replay()
        torch.cuda.synchronize()
        print(f"forward B={B} as {n} concurrent chain(s) of {B // n}: {(time.perf_counter() - t0) / 20 * 1e3:.3f} ms",
              flush=True)


if __name__ == "__main__":
    main()
