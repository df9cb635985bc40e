#!/bin/bash
# Tune only the GEMM shapes the package table has no entry for, per workload (into gpurun_out/tuned_new.json), then
# a same-box A/B of the workloads that gained entries.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
cp stablediffusion-pytorch_amd/sdmi/tuned_gemm.json gpurun_out/tuned_new.json
for W in ${WLS:-cond-unet uncond-unet dit}; do
  timeout -k 10 600 python -u scripts/tune_gemm.py --workload $W --only-new --out gpurun_out/tuned_new.json > gpurun_out/tune_new_$W.log 2>&1 || { tail -30 gpurun_out/tune_new_$W.log; exit 1; }
  echo "$W: $(grep -c 'us  best' gpurun_out/tune_new_$W.log) new shapes"; tail -2 gpurun_out/tune_new_$W.log
done
for SB in 1 8; do
  timeout -k 10 600 python -u scripts/tune_gemm.py --workload sample --sample-batch $SB --only-new --out gpurun_out/tuned_new.json > gpurun_out/tune_new_s$SB.log 2>&1 || { tail -30 gpurun_out/tune_new_s$SB.log; exit 1; }
  echo "sample B=$SB: $(grep -c 'us  best' gpurun_out/tune_new_s$SB.log) new shapes"; tail -2 gpurun_out/tune_new_s$SB.log
done
