#!/bin/bash
# attention round 3: kernel tests, isolated timing and the step A/B of the fused backward (SDMI_ATTN_FUSED) and the
# forward's static softmax offsets (SDMI_ATTN_FIXED); then the diagnostic attribution (gpu_diag.sh)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
SDMI_ATTN_FIXED=1 timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "attention" --timeout 120 --timeout-method thread > gpurun_out/t_attn3.log 2>&1
rc=$?; tail -4 gpurun_out/t_attn3.log; [ $rc -ne 0 ] && exit $rc
for cfg in "SDMI_ATTN_FUSED=0 SDMI_ATTN_FIXED=0" "SDMI_ATTN_FUSED=1 SDMI_ATTN_FIXED=1"; do
  env $cfg timeout -k 10 300 python -u scripts/attn_bench.py > gpurun_out/ab_attn3.txt 2>&1 || { tail -5 gpurun_out/ab_attn3.txt; exit 1; }
  echo "$cfg"; grep "B=" gpurun_out/ab_attn3.txt
done
for i in 1 2; do
  for cfg in "SDMI_ATTN_FUSED=0 SDMI_ATTN_FIXED=0" "SDMI_ATTN_FUSED=0 SDMI_ATTN_FIXED=1" "SDMI_ATTN_FUSED=1 SDMI_ATTN_FIXED=1"; do
    env $cfg timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/b_attn3.log 2>&1 || { tail -20 gpurun_out/b_attn3.log; exit 1; }
    python3 -c "import json;d=json.loads(open('gpurun_out/b_attn3.log').read().strip().splitlines()[-1]);print('$cfg', round(d['ms_per_step'],3), d['last_loss'])"
  done
done
bash scripts/gpu_diag.sh
