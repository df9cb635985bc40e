#!/bin/bash
# attention small-shape G=4 default: kernel + DiT tests, kernel times, cond / DiT steps; GroupNorm backward batch-tail
# cost (rocprofv3 kernel trace of the GN probe with and without dgamma/dbeta)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
ms() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['ms_per_step'],3))" $1; }
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_dit_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_r3d.log 2>&1 || { tail -30 gpurun_out/t_r3d.log; exit 1; }
tail -1 gpurun_out/t_r3d.log
for sh in 6 7 11; do timeout -k 10 100 python -u scripts/attn_bench.py $sh 2>&1 | grep B= || exit 1; done
for G in 2 0; do
  SDMI_ATTN_G=$G timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 30 --workload dit > gpurun_out/dg$G.log 2>&1 || { tail -5 gpurun_out/dg$G.log; exit 1; }
  echo "dit G=$G $(ms gpurun_out/dg$G.log)"
  SDMI_ATTN_G=$G timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 30 > gpurun_out/cg$G.log 2>&1 || { tail -5 gpurun_out/cg$G.log; exit 1; }
  echo "cond G=$G $(ms gpurun_out/cg$G.log)"
done
for T in 0 1; do
  GN_TAIL=$T timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gnt$T -o run -- python3 scripts/gn_tail_probe.py > gpurun_out/gnt$T.log 2>&1 || { tail -5 gpurun_out/gnt$T.log; exit 1; }
done
python3 - <<'PY'
import csv, collections
for T in (0, 1):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f"gpurun_out/gnt{T}/run_kernel_trace.csv")):
        if "gn_bwd" in r["Kernel_Name"]:
            k = (r["Kernel_Name"].split("(")[0][-40:], r.get("Grid_Size_X", r.get("Grid_Size", "")), r.get("Workgroup_Size_X", ""))
            acc[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for k, v in acc.items():
        print("tail", T, k, "n", len(v), "avg us %.2f" % (sum(v[5:]) / max(1, len(v[5:]))))
PY
