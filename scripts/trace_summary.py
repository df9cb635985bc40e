"""Per-kernel time of ONE training step from a rocprofv3 --kernel-trace CSV (true kernel durations,
no host gaps): takes the dispatches between the last two step markers (add_noise), groups them by kernel
name + grid, and prints the groups by total time, plus the step's busy time and idle gaps.
Usage: python scripts/trace_summary.py <run_kernel_trace.csv> [--top 50]"""
import argparse
import csv
import re


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*", "", name)
    return name.replace("void ", "")[:62]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--top", type=int, default=50)
    ap.add_argument("--marker", default="add_noise_kernel",
                    help="kernel name marking one step per occurrence (sampling: ddpm_prev_kernel)")
    args = ap.parse_args()
    rows = list(csv.DictReader(open(args.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # one step marker per step: the noise draw of the step's batch (add_noise_kernel; the gradient norm now runs in
    # several sumsq pieces per step, so it no longer marks steps), the optimizer chunks pipeline into the next forward
    marks = [i for i, r in enumerate(rows) if args.marker in r["Kernel_Name"]]
    if len(marks) < 2:
        raise SystemExit(f"need >= 2 {args.marker} launches (steps) in the trace")
    step = rows[marks[-2] + 1: marks[-1] + 1]
    t0 = int(step[0]["Start_Timestamp"])
    t1 = int(step[-1]["End_Timestamp"])
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in step)
    print(f"step span {(t1 - t0) / 1e6:.3f} ms, kernel busy {busy / 1e6:.3f} ms, {len(step)} dispatches")
    per_stream = {}
    for r in step:
        k = r.get("Stream_Id", r.get("Queue_Id"))
        a = per_stream.setdefault(k, [0, 0])
        a[0] += 1
        a[1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    for k, (c, t) in sorted(per_stream.items(), key=lambda kv: -kv[1][1]):
        print(f"  stream {k}: {c} dispatches, busy {t / 1e6:.3f} ms")
    # union of busy intervals = time at least one kernel runs
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in step)
    union, cs, ce = 0, iv[0][0], iv[0][1]
    for s0, e0 in iv[1:]:
        if s0 > ce:
            union += ce - cs
            cs, ce = s0, e0
        else:
            ce = max(ce, e0)
    union += ce - cs
    print(f"  GPU busy (any stream) {union / 1e6:.3f} ms")
    # phases: from the previous step's gradient norm to the loss = optimizer chunks + packing (side stream) and the
    # forward; from the loss to this step's gradient norm = backward (+ weight gradients on the side stream)
    names = [r["Kernel_Name"] for r in step]
    i_mse = next((i for i, n in enumerate(names) if "mse_kernel" in n), None)
    if i_mse is not None:
        def busy_of(rs, pred=lambda n: True):
            return sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rs if pred(r["Kernel_Name"]))
        opt = lambda n: "adam_ema" in n or "pack" in n  # noqa: E731
        print(f"  phases (kernel busy): forward {busy_of(step[:i_mse], lambda n: not opt(n)) / 1e6:.3f} ms, "
              f"optimizer+pack {busy_of(step, opt) / 1e6:.3f} ms, backward {busy_of(step[i_mse:]) / 1e6:.3f} ms")
    groups = {}
    for r in step:
        wg = int(r["Workgroup_Size_X"])
        grid = (int(r["Grid_Size_X"]) // wg, int(r["Grid_Size_Y"]), int(r["Grid_Size_Z"]))
        key = (short(r["Kernel_Name"]), grid)
        g = groups.setdefault(key, [0, 0])
        g[0] += 1
        g[1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    by_name = {}
    for (n, _), (c, t) in groups.items():
        a = by_name.setdefault(n, [0, 0])
        a[0] += c
        a[1] += t
    print("--- by kernel ---")
    for n, (c, t) in sorted(by_name.items(), key=lambda kv: -kv[1][1]):
        print(f"{t / 1e3:9.1f} us {c:5d}x  avg {t / c / 1e3:7.1f} us  {n}")
    print("--- by kernel + grid (blocks x, y, z) ---")
    for (n, grid), (c, t) in sorted(groups.items(), key=lambda kv: -kv[1][1])[:args.top]:
        print(f"{t / 1e3:9.1f} us {c:4d}x  avg {t / c / 1e3:7.1f} us  {n:62s} grid {grid}")


if __name__ == "__main__":
    main()
