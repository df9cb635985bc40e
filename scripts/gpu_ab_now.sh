#!/bin/bash
# GPU parity suite, then a same-box A/B of the working tree under env settings (scripts/gpu_bisect.sh arms)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 200 --timeout-method thread > gpurun_out/t_ab.log 2>&1
  rc=$?; tail -2 gpurun_out/t_ab.log; [ $rc -eq 0 ] || exit 1
fi
ARMS="${ARMS:-. .:SDMI_TIME_JOIN=1}" bash scripts/gpu_bisect.sh
