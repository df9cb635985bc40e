#!/bin/bash
# Full GPU pass: parity suite, bench line, per-launch profile, rocprofv3 kernel stats of the bench.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-x}
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/t_$TAG.log 2>&1 || { tail -40 gpurun_out/t_$TAG.log; exit 1; }
tail -1 gpurun_out/t_$TAG.log
timeout -k 10 300 python bench.py > gpurun_out/b_$TAG.log 2>&1 || { tail -20 gpurun_out/b_$TAG.log; exit 1; }
tail -1 gpurun_out/b_$TAG.log
timeout -k 10 300 python scripts/profile_step.py --top 45 --dump gpurun_out/ps_all_$TAG.txt > gpurun_out/ps_$TAG.log 2>&1 || { tail -20 gpurun_out/ps_$TAG.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1 || { tail -20 gpurun_out/prof_$TAG.log; exit 1; }
find gpurun_out/prof_$TAG -name "*kernel_stats.csv" | head -1 | xargs -I{} python scripts/kstats.py {} auto
