#!/bin/bash
# Kernel-trace profile of the headline bench: rocprofv3 stats + per-kernel / per-grid trace summary.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-p}
WL=${WL:-cond-unet}
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --workload $WL --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1 || { tail -20 gpurun_out/prof_$TAG.log; exit 1; }
tail -1 gpurun_out/prof_$TAG.log | cut -c1-300
python scripts/trace_summary.py gpurun_out/prof_$TAG/run_kernel_trace.csv --top 60 > gpurun_out/ts_$TAG.txt
head -50 gpurun_out/ts_$TAG.txt
