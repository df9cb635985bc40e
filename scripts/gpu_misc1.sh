#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
A="SDMI_SPLIT_CAP=8" B="SDMI_SPLIT_CAP=24" TAG=cap bash scripts/gpu_ab2.sh || exit 1
timeout -k 10 300 python -u bench.py --workload dit --no-cpu-baseline > gpurun_out/b_dit.log 2>&1 || { tail -20 gpurun_out/b_dit.log; exit 1; }
tail -1 gpurun_out/b_dit.log | cut -c1-300
WL=dit TAG=pdit bash scripts/gpu_prof_r2.sh
