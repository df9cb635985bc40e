#!/bin/bash
# Tune the GEMM table for the sampler's B=1 (and B=8) forward shapes, then bench the captured sampling loop before / after.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
ms() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['ms_per_step'],3))" $1; }
for b in 1 8; do
  timeout -k 10 300 python -u bench.py --workload sample --sample-batch $b --steps 50 --warmup 5 > gpurun_out/smp_before_b$b.log 2>&1 || { tail -5 gpurun_out/smp_before_b$b.log; exit 1; }
  echo "before B=$b $(ms gpurun_out/smp_before_b$b.log)"
done
cp stablediffusion-pytorch_amd/sdmi/tuned_gemm.json gpurun_out/tuned_gemm.json
for b in 1 8; do
  timeout -k 10 900 python -u scripts/tune_gemm.py --workload sample --sample-batch $b --out gpurun_out/tuned_gemm.json > gpurun_out/tune_sample_b$b.txt 2>&1 || { tail -5 gpurun_out/tune_sample_b$b.txt; exit 1; }
  tail -2 gpurun_out/tune_sample_b$b.txt
done
for b in 1 8; do
  SDMI_TUNED_GEMM=gpurun_out/tuned_gemm.json timeout -k 10 300 python -u bench.py --workload sample --sample-batch $b --steps 50 --warmup 5 > gpurun_out/smp_after_b$b.log 2>&1 || { tail -5 gpurun_out/smp_after_b$b.log; exit 1; }
  echo "after B=$b $(ms gpurun_out/smp_after_b$b.log)"
done
