#!/bin/bash
# GEMM mainloop variants: numerics under each forced variant, then the variant probe
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-wg}
for v in ${VARIANTS:-2 4}; do
  SDMI_GEMM_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tg_${TAG}_$v.log 2>&1 || { tail -30 gpurun_out/tg_${TAG}_$v.log; exit 1; }
  tail -1 gpurun_out/tg_${TAG}_$v.log
done
timeout -k 10 400 python -u scripts/variant_probe.py ${PROBE:-1,2,4} > gpurun_out/vp_$TAG.txt 2>&1 || { tail -20 gpurun_out/vp_$TAG.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/vp_$TAG.txt
