"""In-step re-tune of the GEMM table: scripts/tune_gemm.py picks each shape's split count / mainloop in isolation on one
stream, but in the recorded step the forward and data-gradient GEMMs share the chip with the weight-gradient streams.
This re-records the step's plan with one table entry changed at a time and keeps a change only when the WHOLE step,
replayed, is faster (interleaved base / candidate replays in one process, both arms better by > --min-gain ms).

Only row-major launches without reduction columns are touched: the weight-gradient launches with bias / group-sum
columns keep their validated (sample-aligned) entries (the reduction-column path at forced splits).
Writes the table to --out (default gpurun_out/tuned_instep.json), never the package's.
Usage: python scripts/tune_in_step.py [--workload cond-unet] [--keys 14] [--out path]"""
import argparse
import collections
import gc
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "stablediffusion-pytorch_amd"), REPO]
import torch  # noqa: E402

from scripts.device_step import make  # noqa: E402

VARIANTS = (2, 3, 6, 9, 10)


def step_ms(cap, n):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        cap.step()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="cond-unet")
    ap.add_argument("--keys", type=int, default=14)
    ap.add_argument("--steps", type=int, default=15)
    ap.add_argument("--min-gain", type=float, default=0.03)
    ap.add_argument("--out", default=os.path.join(REPO, "gpurun_out", "tuned_instep.json"))
    a = ap.parse_args()
    from sdmi import _lib, kernels as K, streams
    from sdmi.plan import StepPlan
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    streams.reserve(dev, n=streams.workload_streams(a.workload))
    K.GEMM_CAPTURE = []
    cap = make(a.workload, dev)
    descs, K.GEMM_CAPTURE = K.GEMM_CAPTURE, None
    table = K._tuned()
    flops = collections.Counter()
    nkt = {}
    for d in descs:
        if d.a_mode == _lib.A_COLMAJOR or d.sum_out or d.sum_out2 or d.gsum_out:
            continue
        key = K.gemm_key(d)
        flops[key] += 2.0 * d.m * d.n * d.k
        nkt[key] = (d.k + 63) // 64
    keys = [k for k, _ in flops.most_common(a.keys)]
    for _ in range(3):
        cap.step()
    base_plan = cap.plan
    t_start = min(step_ms(cap, a.steps) for _ in range(3))
    print(f"{a.workload}: start {t_start:.3f} ms/step; {len(keys)} keys", flush=True)
    changed = {}
    def put(key, e):
        if e == 0:
            table.pop(key, None)
        else:
            table[key] = e

    for key in keys:
        cur = table.get(key, 0)
        s, v = (cur[0], cur[1]) if isinstance(cur, list) else (cur, 0)
        cands = []
        if s:
            for s2 in (s // 2, s * 2):
                if 1 <= s2 <= min(nkt[key], 16) and s2 != s:
                    cands.append([s2, v])
        for v2 in VARIANTS:
            if v2 != v:
                cands.append([s or 1, v2])
        for cand in cands:
            table[key] = cand
            try:
                plan = StepPlan(cap._run, dev)
            except Exception as e:  # a candidate the library refuses for this shape
                print(f"  {key} {cand}: refused ({e})", flush=True)
                continue
            finally:
                put(key, cur)
            res = []
            for _ in range(2):
                cap.plan = base_plan
                tb = step_ms(cap, a.steps)
                cap.plan = plan
                tc = step_ms(cap, a.steps)
                res.append((tb, tc))
            cap.plan = base_plan
            gains = [tb - tc for tb, tc in res]
            ok = all(g > a.min_gain for g in gains)
            print(f"  {key:58s} {cur} -> {cand}: base {res[0][0]:.3f}/{res[1][0]:.3f} cand {res[0][1]:.3f}/"
                  f"{res[1][1]:.3f}{'  KEEP' if ok else ''}", flush=True)
            if ok:
                cur = cand
                table[key] = cand
                changed[key] = cand
                old, base_plan = base_plan, plan
                cap.plan = base_plan
                del old
            del plan
            gc.collect()
            torch.cuda.empty_cache()
        put(key, cur)
    t_end = min(step_ms(cap, a.steps) for _ in range(3))
    print(f"{a.workload}: {t_start:.3f} -> {t_end:.3f} ms/step; changed {len(changed)}: {changed}", flush=True)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(dict(sorted(table.items())), f, indent=0)
    print("wrote", a.out)


if __name__ == "__main__":
    main()
