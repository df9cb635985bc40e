#!/bin/bash
# in-launch split-K combine (last-arriving split sums the tile's slabs; now for every tile shape incl. the 64-row
# 6-stage variants): GEMM / B=32 step parity with it forced on, then the step A/B over SDMI_SPLITK_FUSED caps
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
SDMI_SPLITK_FUSED=128 timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_bench_step_gpu.py tests/test_plan_gpu.py -q -x --timeout 200 --timeout-method thread > gpurun_out/t_skf.log 2>&1
rc=$?; tail -2 gpurun_out/t_skf.log; [ $rc -eq 0 ] || exit 1
AB_TESTS=0 bash scripts/gpu_ab_full.sh
