#!/bin/bash
# Sampling with the per-run context cache: sampling tests, then bench B = 1 / 8 (DDPM) and DDIM B = 1, alternating the
# cache on / off (SDMI_SAMPLE_CTX_CACHE) on the same box
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
ms() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['ms_per_step'],3))" $1; }
timeout -k 10 300 python -u -m pytest tests/test_sampling_gpu.py tests/test_module_gpu.py -q --timeout 200 --timeout-method thread > gpurun_out/t_r3h.log 2>&1 || { tail -30 gpurun_out/t_r3h.log; exit 1; }
tail -1 gpurun_out/t_r3h.log
for r in 1 2; do
  for B in 1 8; do
    timeout -k 10 200 python -u bench.py --workload sample --sample-batch $B --steps 40 --no-cpu-baseline > gpurun_out/s.log 2>&1 || { tail -20 gpurun_out/s.log; exit 1; }
    cp gpurun_out/s.log gpurun_out/bs${B}_r3h.log
    echo "B=$B new $(ms gpurun_out/s.log)"
    SDMI_SAMPLE_CTX_CACHE=0 timeout -k 10 200 python -u bench.py --workload sample --sample-batch $B --steps 40 --no-cpu-baseline > gpurun_out/s.log 2>&1 || { tail -20 gpurun_out/s.log; exit 1; }
    echo "B=$B no-cache $(ms gpurun_out/s.log)"
  done
done
timeout -k 10 300 python -u bench.py --workload sample --sampler ddim --steps 50 --no-cpu-baseline > gpurun_out/bsd_r3h.log 2>&1 || { tail -20 gpurun_out/bsd_r3h.log; exit 1; }
echo "ddim B=1 $(ms gpurun_out/bsd_r3h.log)"
