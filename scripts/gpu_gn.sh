#!/bin/bash
# GroupNorm change check: kernel + model parity tests, then A/B of the headline bench (legacy single-pass shape vs new)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-gn}
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_unet_gpu.py tests/test_plan_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1 || { tail -30 gpurun_out/t_$TAG.log; exit 1; }
tail -2 gpurun_out/t_$TAG.log
A="${GA:-SDMI_X=0}" B="${GB:-SDMI_GN_LEGACY=1}" TAG=$TAG bash scripts/gpu_ab2.sh
