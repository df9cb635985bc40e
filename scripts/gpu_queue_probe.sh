#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for C in order reverse rccl rccl_reverse cumask rccl_cumask; do
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/qp_$C -o run -- python3 scripts/queue_probe.py $C > gpurun_out/qp_$C.log 2>&1 || { tail -20 gpurun_out/qp_$C.log; exit 1; }
  python3 - gpurun_out/qp_$C $C <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
print(sys.argv[2], " ".join(f"s{r['Stream_Id']}:q{r['Queue_Id']}:{r['Kernel_Name'][:18]}:{r['Grid_Size_X']}" for r in rows))
PY
done
