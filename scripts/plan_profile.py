"""Isolated device time of every kernel of one recorded training step (the native plan's launches re-issued one at a
time on their own buffers, sdmi_plan_time_op), GEMMs labelled with their shapes and rates, plus the vendor library
(hipBLASLt via torch.matmul) on the same plain GEMM shapes as a yardstick.
Usage: python scripts/plan_profile.py [--workload cond-unet|dit|uncond-unet] [--top 60]"""
import argparse
import ctypes
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "stablediffusion-pytorch_amd"), REPO]
import torch  # noqa: E402

import bench  # noqa: E402
from scripts.device_step import make  # noqa: E402


# PLAN_PROFILE_ITERS="warm,iters" (default 2,10); "0,1" re-issues every launch exactly once, for rocprofv3 --pmc
# passes whose per-dispatch counters are then each launch measured alone (scripts/gpu_pmc_isolated.sh)
WARM, ITERS = (int(v) for v in os.environ.get("PLAN_PROFILE_ITERS", "2,10").split(","))


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="cond-unet")
    ap.add_argument("--top", type=int, default=70)
    a = ap.parse_args()
    from sdmi import kernels as K, _lib
    from sdmi.plan import StepPlan
    dev = torch.device("cuda", 0)
    K.GEMM_LOG = []
    cap = make(a.workload, dev)  # warm-up steps + the recorded step all log; keep the recorded step's calls
    log = K.GEMM_LOG
    K.GEMM_LOG = None
    per_step = len(log) // 3
    log = log[-per_step:]
    plan = cap.plan
    lib = _lib.lib()
    n, nl, nc = plan.info()
    ops = []
    kind, name, grid, block, shm = (ctypes.c_int(), ctypes.c_char_p(), (ctypes.c_int * 3)(), ctypes.c_int(),
                                    ctypes.c_int())
    for i in range(n):
        _lib.check(lib.sdmi_plan_op_info(plan.handle, i, ctypes.byref(kind), ctypes.byref(name), grid,
                                         ctypes.byref(block), ctypes.byref(shm)), "op_info")
        if kind.value != 0:
            continue
        us = ctypes.c_float()
        _lib.check(lib.sdmi_plan_time_op(plan.handle, i, WARM, ITERS, ctypes.byref(us)), "time_op")
        ops.append(dict(i=i, name=name.value.decode(errors="replace") if name.value else "?", grid=tuple(grid),
                        us=us.value))
    dem = subprocess.run(["c++filt"], input="\n".join(o["name"] for o in ops), capture_output=True, text=True).stdout
    for o, nm in zip(ops, dem.splitlines()):
        o["name"] = nm.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
    torch.cuda.synchronize()
    # attach GEMM shapes in issue order
    gi = 0
    for j, op in enumerate(ops):
        if op["name"].startswith("gemm") and gi < len(log):
            op["gemm"] = log[gi]
            if log[gi]["splits"] > 1 and j + 1 < len(ops) and ops[j + 1]["name"].startswith("splitk_reduce"):
                ops[j + 1]["reduce_of"] = log[gi]
            gi += 1
    total = sum(o["us"] for o in ops)
    if os.environ.get("PLAN_PROFILE_JSON"):
        import json
        json.dump([dict(i=o["i"], name=o["name"], grid=o["grid"], us=o["us"], gemm=o.get("gemm"),
                        reduce=o.get("reduce_of") is not None) for o in ops],
                  open(os.environ["PLAN_PROFILE_JSON"], "w"))
    print(f"{a.workload}: {n} ops, {nl} launches, {nc} callouts; isolated kernel time {total / 1e3:.2f} ms "
          f"(GEMM calls matched {gi}/{len(log)})")
    fam = {}
    for o in ops:
        f = fam.setdefault(o["name"][:62], [0.0, 0])
        f[0] += o["us"]
        f[1] += 1
    print("--- by kernel (isolated) ---")
    for nm, (t, c) in sorted(fam.items(), key=lambda kv: -kv[1][0])[:30]:
        print(f"  {t:9.1f} us {c:4d}x  {nm}")
    print("--- GEMM shapes by total isolated time (us incl. its split-K reducer; TF = 2MNK / time) ---")
    shapes = {}
    for j, o in enumerate(ops):
        gm = o.get("gemm")
        if gm is None:
            continue
        t = o["us"] + (ops[j + 1]["us"] if j + 1 < len(ops) and ops[j + 1].get("reduce_of") is gm else 0.0)
        key = (gm["a"], gm["b"], gm["m"], gm["n"], gm["k"], gm["conv"], gm["splits"], gm["tile_n"], gm["phase"],
               o["grid"])
        s = shapes.setdefault(key, [0.0, 0, gm["flops"]])
        s[0] += t
        s[1] += 1
    rows = sorted(shapes.items(), key=lambda kv: -kv[1][0])
    for key, (t, c, fl) in rows[:a.top]:
        aa, bb, m, nn, kk, conv, sp, tn, ph, gr = key
        print(f"  {t:8.1f} us {c:3d}x  a{aa}b{bb} {ph:>3s} M={m:6d} N={nn:5d} K={kk:6d} conv={conv} split={sp:2d} "
              f"tile={tn} grid={gr}  {fl * c / (t * 1e-6) / 1e12:6.1f} TF")
    if os.environ.get("PLAN_PROFILE_NO_BLAS"):
        return
    # vendor yardstick on the plain (non-conv) GEMM shapes
    print("--- hipBLASLt (torch.matmul, bf16) on the same plain shapes ---")
    seen = set()
    for key, (t, c, fl) in rows:
        aa, bb, m, nn, kk, conv, sp, tn, ph, gr = key
        if aa == 1 or bb == 2 or (aa, bb, m, nn, kk) in seen:
            continue
        seen.add((aa, bb, m, nn, kk))
        A = torch.randn(m, kk, device=dev, dtype=torch.bfloat16) if aa == 0 else \
            torch.randn(kk, m, device=dev, dtype=torch.bfloat16).t()
        Bm = torch.randn(nn, kk, device=dev, dtype=torch.bfloat16).t() if bb == 0 else \
            torch.randn(kk, nn, device=dev, dtype=torch.bfloat16)
        us = timeit(lambda: torch.matmul(A, Bm))
        print(f"  a{aa}b{bb} M={m:6d} N={nn:5d} K={kk:6d}: ours {t / c:7.1f} us/launch, hipBLASLt {us:7.1f} us "
              f"({2 * m * nn * kk / (us * 1e-6) / 1e12:6.1f} TF)")
        if len(seen) >= 25:
            break


if __name__ == "__main__":
    main()
