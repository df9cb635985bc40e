#!/bin/bash
# attention kernels: isolated timings at the step shapes + rocprofv3 per-kernel stats (fwd / dq / dkv split)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-at}
timeout -k 10 120 python -u scripts/attn_bench.py > gpurun_out/attn_$TAG.log 2>&1 || { tail -20 gpurun_out/attn_$TAG.log; exit 1; }
cat gpurun_out/attn_$TAG.log | grep -v amdgpu.ids
for i in 0 1; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/aprof_${TAG}_$i -o run -- python3 scripts/attn_bench.py $i > /dev/null 2>&1 || { echo "rocprof $i failed"; exit 1; }
  python3 - "$i" <<PY
import csv, sys
rows = list(csv.DictReader(open("gpurun_out/aprof_${TAG}_%s/run_kernel_stats.csv" % sys.argv[1])))
for r in rows:
    if "attn" in r["Name"]:
        print(sys.argv[1], r["Name"][:40], r["Calls"], "avg us", round(float(r["AverageNs"]) / 1e3, 1))
PY
done
