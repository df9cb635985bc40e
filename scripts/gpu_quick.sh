#!/bin/bash
# Quick GPU pass: GEMM numerics, then bench (graph) and the per-launch profile.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-q}
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/t_$TAG.log 2>&1 || { tail -40 gpurun_out/t_$TAG.log; exit 1; }
tail -1 gpurun_out/t_$TAG.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/b_$TAG.log 2>&1 || { tail -20 gpurun_out/b_$TAG.log; exit 1; }
tail -1 gpurun_out/b_$TAG.log | cut -c1-300
timeout -k 10 300 python bench.py --no-cpu-baseline --graph 2>&1 | tail -1 | cut -c1-300
SDMI_WG_STREAM=0 timeout -k 10 300 python bench.py --no-cpu-baseline 2>&1 | tail -1 | cut -c1-300
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr_$TAG -o run -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/tr_$TAG.log 2>&1 || { tail -20 gpurun_out/tr_$TAG.log; exit 1; }
python scripts/trace_summary.py gpurun_out/tr_$TAG/run_kernel_trace.csv --top 40 > gpurun_out/ts_$TAG.txt
head -24 gpurun_out/ts_$TAG.txt
