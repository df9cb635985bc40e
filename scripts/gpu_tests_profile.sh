#!/bin/bash
# the GPU suite, then the closing profile of the headline step (scripts/gpu_profile.sh) under TAG
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/t_$TAG.log; [ $rc -eq 0 ] || exit 1
bash scripts/gpu_profile.sh
