"""Per-kernel time of ONE training step from a rocprofv3 --kernel-trace CSV (true kernel durations,
no host gaps): takes the dispatches between the last two optimizer launches, groups them by kernel
name + grid, and prints the groups by total time, plus the step's busy time and idle gaps.
Usage: python scripts/trace_summary.py <run_kernel_trace.csv> [--top 50]"""
import argparse
import csv
import re


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*", "", name)
    return name.replace("void ", "")[:48]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--top", type=int, default=50)
    args = ap.parse_args()
    rows = list(csv.DictReader(open(args.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if "adam_ema_kernel" in r["Kernel_Name"]]
    if len(marks) < 2:
        raise SystemExit("need >= 2 optimizer launches in the trace")
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
    # phases on the issuing stream: forward = before the loss kernel, backward, optimizer = from sumsq on
    names = [r["Kernel_Name"] for r in step]
    i_mse = next((i for i, n in enumerate(names) if "mse_kernel" in n), None)
    i_opt = next((i for i, n in enumerate(names) if "sumsq_kernel" in n), None)
    if i_mse is not None and i_opt is not None:
        def span_busy(a, b):
            return sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in step[a:b])
        print(f"  phases (kernel busy): forward {span_busy(0, i_mse) / 1e6:.3f} ms, "
              f"backward {span_busy(i_mse, i_opt) / 1e6:.3f} ms, optimizer+pack {span_busy(i_opt, len(step)) / 1e6:.3f} ms")
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
        print(f"{t / 1e3:9.1f} us {c:4d}x  avg {t / c / 1e3:7.1f} us  {n:40s} grid {grid}")


if __name__ == "__main__":
    main()
