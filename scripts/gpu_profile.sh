#!/bin/bash
# Round profile: bench line + rocprofv3 kernel trace/stats of the same bench command (files under gpurun_out/).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r01}
timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
tail -1 gpurun_out/bench_$TAG.json | cut -c1-200
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o bench -- python3 bench.py --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1 || { tail -20 gpurun_out/prof_$TAG.log; exit 1; }
tail -1 gpurun_out/prof_$TAG.log | cut -c1-200
python scripts/trace_summary.py gpurun_out/prof_$TAG/bench_kernel_trace.csv --top 60 > gpurun_out/ts_$TAG.txt
python scripts/kstats.py gpurun_out/prof_$TAG/bench_kernel_stats.csv auto > gpurun_out/ks_$TAG.txt
head -12 gpurun_out/ts_$TAG.txt
