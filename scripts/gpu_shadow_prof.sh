#!/bin/bash
# Why SDMI_SHADOW=1 measured slower: isolated per-launch plan profile and an in-step kernel trace for both settings;
# plus the leaf-glue kernel tests.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_leafops_gpu.py tests/test_leaf_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_leafops.log 2>&1
rc=$?; tail -3 gpurun_out/t_leafops.log; [ $rc -eq 0 ] || exit 1
for sh in 0 1; do
  SDMI_SHADOW=$sh timeout -k 10 400 python -u scripts/plan_profile.py --top 40 > gpurun_out/pp_sh$sh.txt 2>&1 || { tail -20 gpurun_out/pp_sh$sh.txt; exit 1; }
  head -24 gpurun_out/pp_sh$sh.txt
  SDMI_SHADOW=$sh timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_sh$sh -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof_sh$sh.log 2>&1 || { tail -20 gpurun_out/prof_sh$sh.log; exit 1; }
  python scripts/trace_summary.py gpurun_out/prof_sh$sh/run_kernel_trace.csv --top 40 > gpurun_out/ts_sh$sh.txt
  head -30 gpurun_out/ts_sh$sh.txt
done
