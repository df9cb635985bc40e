#!/bin/bash
# gemm.hip without SLP packing + attention occupancy variants: kernel tests, the occupancy sweep at the 32^2 / 16^2
# shapes, then the step A/B against ab_old/ (new = occupancy 2, new+env = the AB_ENV_NEW occupancy)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_gemm_gpu.py tests/test_plan_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/t_r3b.log 2>&1
rc=$?; tail -2 gpurun_out/t_r3b.log; [ $rc -eq 0 ] || exit 1
for cfg in "SDMI_ATTN_OCC_FWD=2 SDMI_ATTN_OCC_DQ=2 SDMI_ATTN_OCC_DKV=2" "SDMI_ATTN_OCC_FWD=3 SDMI_ATTN_OCC_DQ=3 SDMI_ATTN_OCC_DKV=3" "SDMI_ATTN_OCC_FWD=4 SDMI_ATTN_OCC_DQ=3 SDMI_ATTN_OCC_DKV=2"; do
  echo "== $cfg"
  for i in 0 2 6; do
    env $cfg timeout -k 10 120 python -u scripts/attn_bench.py $i > gpurun_out/occ.txt 2>&1 && grep "B=" gpurun_out/occ.txt
  done
done
AB_TESTS=0 bash scripts/gpu_ab_full.sh
