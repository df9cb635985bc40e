"""Per-dispatch PMC counter values of the kernels whose name contains a pattern (last dispatch of each kernel).
Usage: python scripts/pmc_kernel.py <run_counter_collection.csv> <name-substring>"""
import collections
import csv
import sys


def main():
    path, pat = sys.argv[1], sys.argv[2]
    agg = collections.defaultdict(float)
    names = {}
    for r in csv.DictReader(open(path)):
        if pat not in r["Kernel_Name"]:
            continue
        agg[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        names[r["Dispatch_Id"]] = r["Kernel_Name"][:60]
    last = {}
    for (d, c), v in sorted(agg.items(), key=lambda kv: int(kv[0][0])):
        last[(names[d], c)] = v
    for (n, c), v in sorted(last.items()):
        print(f"{n:60s} {c:28s} {v:16.0f}")


if __name__ == "__main__":
    main()
