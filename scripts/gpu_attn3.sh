#!/bin/bash
# fused attention backward: kernel tests, then isolated timing fused vs two-kernel, then the step A/B
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -q -x -k attention --timeout 120 --timeout-method thread > gpurun_out/t_attn3.log 2>&1
rc=$?; tail -4 gpurun_out/t_attn3.log; [ $rc -ne 0 ] && exit $rc
for f in 0 1; do
  SDMI_ATTN_FUSED=$f timeout -k 10 300 python -u scripts/attn_bench.py > gpurun_out/ab_attn3_$f.txt 2>&1 || { tail -5 gpurun_out/ab_attn3_$f.txt; exit 1; }
  echo "fused=$f"; grep "B=" gpurun_out/ab_attn3_$f.txt
done
for i in 1 2; do
  for f in 0 1; do
    SDMI_ATTN_FUSED=$f timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/b_attn3_$f$i.log 2>&1 || { tail -20 gpurun_out/b_attn3_$f$i.log; exit 1; }
    python3 -c "import json;d=json.loads(open('gpurun_out/b_attn3_$f$i.log').read().strip().splitlines()[-1]);print('fused=$f', d['ms_per_step'], d['last_loss'])"
  done
done
bash scripts/gpu_diag.sh
