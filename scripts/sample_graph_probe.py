"""Probe: the captured DDPM sampling step replayed as a native launch plan (sdmi.plan) vs as one hipGraph
(torch.cuda.CUDAGraph of the same eager step), at B = argv[1]: ms per reverse step, host enqueue time per step,
and bitwise equality of x_t after K steps from the same start. Run once with SDMI_CTX_STREAM=0 (single stream)
and once with the default context stream."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "stablediffusion-pytorch_amd"))

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    os.environ["SDMI_SAMPLE_ISSUE"] = "plan"  # the loop records a plan; the graph below is captured here
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    K = 20
    dev = torch.device("cuda", 0)
    import models.unet_cond_base as mc
    from scheduler.linear_noise_scheduler import LinearNoiseScheduler
    from sdmi.sampling import DDPMSampleLoop
    cfg = bench.cond_config()
    torch.manual_seed(1111)
    model = mc.Unet(4, cfg).to(dev).eval()
    x0, text, empty, mask = bench.synthetic_batch(B, dev, 1111)
    sched = LinearNoiseScheduler(1000, 0.00085, 0.012)
    loop = DDPMSampleLoop(model, sched, (B, 4, 32, 32), cond_input={"text": text, "image": mask}, seed=0)
    xT = torch.randn(B, 4, 32, 32, generator=torch.Generator().manual_seed(5)).to(dev)

    # plan: record on the first step, then replay
    loop.run(xT, steps=3, captured=True)
    torch.cuda.synchronize()
    loop.reset(xT)
    for _ in range(K):
        loop.plan.replay()
    torch.cuda.synchronize()
    ref = loop.xt.clone()
    loop.reset(xT)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(K):
        loop.plan.replay()
    th = time.perf_counter() - t0
    torch.cuda.synchronize()
    tp = time.perf_counter() - t0
    print(f"B={B} ctx_stream={os.environ.get('SDMI_CTX_STREAM', '1')} plan: {tp / K * 1e3:.3f} ms/step, host "
          f"enqueue {th / K * 1e3:.3f} ms/step", flush=True)

    # graph of the eager step
    loop.reset(xT)
    s = torch.cuda.Stream(device=dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        loop._step()
    torch.cuda.current_stream(dev).wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        loop._step()
    torch.cuda.synchronize()
    loop.reset(xT)
    for _ in range(K):
        g.replay()
    torch.cuda.synchronize()
    same = torch.equal(loop.xt, ref)
    loop.reset(xT)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(K):
        g.replay()
    th = time.perf_counter() - t0
    torch.cuda.synchronize()
    tg = time.perf_counter() - t0
    print(f"B={B} ctx_stream={os.environ.get('SDMI_CTX_STREAM', '1')} graph: {tg / K * 1e3:.3f} ms/step, host "
          f"enqueue {th / K * 1e3:.3f} ms/step, bitwise equal to plan after {K} steps: {same}", flush=True)


if __name__ == "__main__":
    main()
