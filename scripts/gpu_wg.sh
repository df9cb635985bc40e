#!/bin/bash
# weight-gradient / MN-contiguous GEMM variants: numerics under each forced mainloop, then the probe
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-wg}
for v in 2 3; do
  SDMI_GEMM_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tg_${TAG}_$v.log 2>&1 || { tail -30 gpurun_out/tg_${TAG}_$v.log; exit 1; }
  tail -1 gpurun_out/tg_${TAG}_$v.log
done
for v in 0 2 3; do
  SDMI_GEMM_VARIANT=$v SPLITS=${SPLITS:-1,4,8,16,32} timeout -k 10 200 python -u scripts/wgrad_probe.py > gpurun_out/wg_${TAG}_$v.txt 2>&1 || { tail -20 gpurun_out/wg_${TAG}_$v.txt; exit 1; }
  echo "variant $v"; cat gpurun_out/wg_${TAG}_$v.txt | grep -v amdgpu.ids
done
