#!/bin/bash
# GPU suite (-x), the bf16-wire rehearsal kernel traces (1 vs 3 steps), the isolated-plan
# PMC traffic, then the bench line.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/t_dp.log 2>&1
rc=$?; tail -4 gpurun_out/t_dp.log; [ $rc -eq 0 ] || exit 1
for S in 1 3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/wire_$S -o run -- python3 scripts/wire_rehearsal.py $S bf16 > gpurun_out/wire_$S.log 2>&1 || { tail -5 gpurun_out/wire_$S.log; exit 1; }
  tail -1 gpurun_out/wire_$S.log
done
TAG=r04 bash scripts/gpu_pmc_isolated.sh || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/b_dp.log 2>&1 || { tail -5 gpurun_out/b_dp.log; exit 1; }
tail -1 gpurun_out/b_dp.log | cut -c1-300
