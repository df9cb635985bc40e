"""rocprofv3 evidence for bench.py's `roofline` kernel, restricted to the launches the bench's HIP events time:
the UNSPLIT launches (grid z == 1; split-K launches are excluded there because their event also brackets the
reducer). From a --kernel-trace CSV (or a directory holding one): average duration of those launches; from the
--pmc FETCH_SIZE / WRITE_SIZE passes (each run with --kernel-trace as well, so every counter row joins its own
dispatch's per-axis grid by Dispatch_Id): HBM bytes per unsplit launch (FETCH_SIZE x2, the gfx950 correction of
MI355X_MICROARCH.md's HBM section; both counters in KiB).

--tail-frac F keeps only the last fraction F of the kernel's dispatches in each file (the isolated-plan passes of
scripts/gpu_pmc_isolated.sh: 3 step executions while the plan is recorded, then every launch re-issued alone once -> 0.25).

--launches all: every launch of the kernel (split-K ones included: the bench times those with their reducer when the
kernel's unsplit launches carry less than half its work, roofline.launch_set).
--meta WORKLOAD DIGEST: recorded as _meta (bench.py matches DIGEST against the running tree's sdmi._build.source_digest).

Usage: python scripts/roofline_evidence.py <kernel_trace.csv|dir> <fetch_dir> <write_dir> "<kernel>" [--json out]
       [--tail-frac F] [--launches unsplit|all] [--meta WORKLOAD DIGEST]"""
import csv
import glob
import json
import os
import sys


def _trace_csv(p):
    if os.path.isdir(p):
        return glob.glob(os.path.join(p, "**", "*kernel_trace.csv"), recursive=True)[0]
    return p


def _grid_z(d):
    """Dispatch_Id -> grid z of the pass's own kernel trace"""
    return {r["Dispatch_Id"]: int(r["Grid_Size_Z"]) for r in csv.DictReader(open(_trace_csv(d)))}


def _match(kernel, name):
    """bench.py's kernel_name() glob (e.g. gemm_dma_kernel<2, 2, 2, 128, 128, 2, *, 64, *, 1>) vs a demangled name"""
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import kernel_matches
    return kernel_matches(kernel, name)


def _tail(rows, frac):
    return rows[len(rows) - int(round(len(rows) * frac)):] if frac < 1.0 else rows


def main():
    trace, fdir, wdir, kernel = sys.argv[1:5]
    frac = float(sys.argv[sys.argv.index("--tail-frac") + 1]) if "--tail-frac" in sys.argv else 1.0
    launches = sys.argv[sys.argv.index("--launches") + 1] if "--launches" in sys.argv else "unsplit"
    keep = (lambda z: z == 1) if launches == "unsplit" else (lambda z: z is not None)
    durs = []
    rows = sorted((r for r in csv.DictReader(open(_trace_csv(trace))) if _match(kernel, r["Kernel_Name"])),
                  key=lambda r: int(r["Dispatch_Id"]))
    for r in _tail(rows, frac):
        if keep(int(r["Grid_Size_Z"])):
            durs.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    out = {"kernel": kernel, "launches": launches, "trace_launches": len(durs),
           "trace_avg_us": sum(durs) / len(durs) if durs else None}
    for d, cname, mul in ((fdir, "FETCH_SIZE", 2.0), (wdir, "WRITE_SIZE", 1.0)):
        vals = []
        gz = _grid_z(d)
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            rows = sorted((r for r in csv.DictReader(open(f))
                           if r["Counter_Name"] == cname and _match(kernel, r["Kernel_Name"])),
                          key=lambda r: int(r["Dispatch_Id"]))
            for r in _tail(rows, frac):
                if keep(gz.get(r["Dispatch_Id"])):
                    vals.append(float(r["Counter_Value"]) * 1024 * mul)
        out[cname.lower() + "_bytes_per_launch"] = sum(vals) / len(vals) if vals else None
        out[cname.lower() + "_launches"] = len(vals)
    if out["fetch_size_bytes_per_launch"] is not None and out["write_size_bytes_per_launch"] is not None:
        out["traffic_bytes_per_launch"] = out["fetch_size_bytes_per_launch"] + out["write_size_bytes_per_launch"]
    if "--meta" in sys.argv:
        i = sys.argv.index("--meta")
        out["_meta"] = {"workload": sys.argv[i + 1], "source_digest": sys.argv[i + 2]}
    print(json.dumps(out, indent=1))
    if "--json" in sys.argv:
        json.dump(out, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
