#!/bin/bash
# Re-tune the GEMM table on the current tree (the GEMM-natural conv weight gradients are new keys, p0) for the
# cond-UNet and DiT steps, then A/B the steps with the new table against the committed one (same box)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
ms() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['ms_per_step'],3))" $1; }
cp stablediffusion-pytorch_amd/sdmi/tuned_gemm.json gpurun_out/tuned_gemm.json
timeout -k 10 900 python -u scripts/tune_gemm.py --workload cond-unet --out gpurun_out/tuned_gemm.json > gpurun_out/tune_cond_r3b.txt 2>&1 || { tail -5 gpurun_out/tune_cond_r3b.txt; exit 1; }
tail -2 gpurun_out/tune_cond_r3b.txt
timeout -k 10 900 python -u scripts/tune_gemm.py --workload dit --out gpurun_out/tuned_gemm.json > gpurun_out/tune_dit_r3b.txt 2>&1 || { tail -5 gpurun_out/tune_dit_r3b.txt; exit 1; }
tail -2 gpurun_out/tune_dit_r3b.txt
for r in 1 2; do
  for W in cond-unet dit; do
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 30 --workload $W > gpurun_out/rt.log 2>&1 || { tail -5 gpurun_out/rt.log; exit 1; }
    echo "$W committed-table $(ms gpurun_out/rt.log)"
    SDMI_TUNED_GEMM=gpurun_out/tuned_gemm.json timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 30 --workload $W > gpurun_out/rt.log 2>&1 || { tail -5 gpurun_out/rt.log; exit 1; }
    echo "$W new-table $(ms gpurun_out/rt.log)"
  done
done
