#!/bin/bash
# Epilogue prefetch A/B: GEMM numerics, the epilogue probe, then cond-UNet and DiT steps alternating
# SDMI_EPI_PREFETCH=0 / 1 on one box.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
ms() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['ms_per_step'],3))" $1; }
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_epi.log 2>&1 || { tail -30 gpurun_out/t_epi.log; exit 1; }
tail -1 gpurun_out/t_epi.log
SDMI_EPI_PREFETCH=0 timeout -k 10 150 python -u scripts/epi_probe.py > gpurun_out/epi0.log 2>&1 || exit 1
timeout -k 10 150 python -u scripts/epi_probe.py > gpurun_out/epi1.log 2>&1 || exit 1
for r in 1 2; do
  for p in 0 1; do
    SDMI_EPI_PREFETCH=$p timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 30 > gpurun_out/c$p.log 2>&1 || { tail -5 gpurun_out/c$p.log; exit 1; }
    echo "cond pre=$p $(ms gpurun_out/c$p.log)"
  done
done
for p in 0 1; do
  SDMI_EPI_PREFETCH=$p timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 30 --workload dit > gpurun_out/d$p.log 2>&1 || { tail -5 gpurun_out/d$p.log; exit 1; }
  echo "dit pre=$p $(ms gpurun_out/d$p.log)"
done
