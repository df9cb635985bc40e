#!/bin/bash
# attention occupancy variants (__launch_bounds__ minimum workgroups per CU) at the model's shapes, then the step
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "attention" --timeout 120 --timeout-method thread > gpurun_out/t_occ.log 2>&1
rc=$?; tail -2 gpurun_out/t_occ.log; [ $rc -eq 0 ] || exit 1
for cfg in "SDMI_ATTN_OCC_FWD=2 SDMI_ATTN_OCC_DQ=2 SDMI_ATTN_OCC_DKV=2" "SDMI_ATTN_OCC_FWD=3 SDMI_ATTN_OCC_DQ=3 SDMI_ATTN_OCC_DKV=3" "SDMI_ATTN_OCC_FWD=4 SDMI_ATTN_OCC_DQ=3 SDMI_ATTN_OCC_DKV=3"; do
  echo "== $cfg"
  env $cfg SDMI_ATTN_OCC_FWD_ONLY=1 timeout -k 10 120 python -u scripts/attn_bench.py 0 > gpurun_out/occ.txt 2>&1 && grep "B=" gpurun_out/occ.txt
  env $cfg timeout -k 10 120 python -u scripts/attn_bench.py 2 > gpurun_out/occ.txt 2>&1 && grep "B=" gpurun_out/occ.txt
  env $cfg timeout -k 10 120 python -u scripts/attn_bench.py 6 > gpurun_out/occ.txt 2>&1 && grep "B=" gpurun_out/occ.txt
done
