#!/bin/bash
# Attention backward rows-per-wave A/B (SDMI_ATTN_G=2 / 4): kernel tests under both, isolated kernel times at the
# 32^2 shapes, then the cond-UNet step alternating.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
ms() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['ms_per_step'],3))" $1; }
for G in 2 4; do
  SDMI_ATTN_G=$G timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k attention --timeout 120 --timeout-method thread > gpurun_out/t_g$G.log 2>&1 || { tail -30 gpurun_out/t_g$G.log; exit 1; }
  echo "G=$G $(tail -1 gpurun_out/t_g$G.log)"
done
for G in 2 4; do
  for sh in 0 1 2 6 7; do SDMI_ATTN_G=$G timeout -k 10 100 python -u scripts/attn_bench.py $sh 2>&1 | grep B= | sed "s/^/G=$G /" || exit 1; done
done
for r in 1 2; do
  for G in 2 4; do
    SDMI_ATTN_G=$G timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 30 > gpurun_out/cg$G.log 2>&1 || { tail -5 gpurun_out/cg$G.log; exit 1; }
    echo "cond G=$G $(ms gpurun_out/cg$G.log)"
  done
done
