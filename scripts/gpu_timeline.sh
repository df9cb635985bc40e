#!/bin/bash
# host issue time of a replayed step + device-true kernel timeline of 2 steps (scripts/device_step.py) under rocprofv3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-tl}
WL=${WL:-cond-unet}
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -q --timeout 300 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1
  tail -4 gpurun_out/t_$TAG.log
fi
timeout -k 10 200 python -u scripts/device_step.py --workload $WL --timeline-steps 0 > gpurun_out/ds_$TAG.log 2>&1 || { tail -20 gpurun_out/ds_$TAG.log; exit 1; }
cat gpurun_out/ds_$TAG.log | grep -v amdgpu.ids
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl_$TAG -o run -- python3 scripts/device_step.py --workload $WL > gpurun_out/tlr_$TAG.log 2>&1 || { tail -20 gpurun_out/tlr_$TAG.log; exit 1; }
grep timeline gpurun_out/tlr_$TAG.log
python scripts/critical_path.py gpurun_out/tl_$TAG/run_kernel_trace.csv --gaps ${GAPS:-20} > gpurun_out/cp_$TAG.txt
python scripts/trace_summary.py gpurun_out/tl_$TAG/run_kernel_trace.csv --top 60 > gpurun_out/ts_$TAG.txt
head -30 gpurun_out/cp_$TAG.txt
