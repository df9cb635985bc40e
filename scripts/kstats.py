"""Summarise a rocprofv3 --stats kernel_stats.csv: per-kernel ms per step.
Usage: python scripts/kstats.py <kernel_stats.csv> <steps_profiled | auto>"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
arg = sys.argv[2] if len(sys.argv) > 2 else "auto"
if arg == "auto":  # one optimizer launch per step
    steps = float(sum(int(r["Calls"]) for r in rows if "adam_ema_kernel" in r["Name"]))
else:
    steps = float(arg)
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total kernel time per step: {tot / 1e6 / steps:.3f} ms")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:30]:
    name = r["Name"].replace("(anonymous namespace)::", "")
    print(f"{float(r['TotalDurationNs']) / 1e6 / steps:8.3f} ms/step {int(r['Calls']) / steps:7.1f}/step "
          f"avg {float(r['AverageNs']) / 1e3:8.1f} us  {name[:90]}")
