#!/bin/bash
# the 64 x 128 three- / two-stage mainloops (variants 9, 10) tried against the current table's entry of every GEMM of the
# cond-UNet and DiT steps, then the headline and DiT bench with the updated table vs the package's (same box)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
cp stablediffusion-pytorch_amd/sdmi/tuned_gemm.json gpurun_out/tuned_v910.json
for WL in cond-unet dit; do
  SDMI_TUNE_VARIANTS=9,10 timeout -k 10 600 python -u scripts/tune_gemm.py --workload $WL --against-table --out gpurun_out/tuned_v910.json > gpurun_out/tune_v910_$WL.log 2>&1 || { tail -5 gpurun_out/tune_v910_$WL.log; exit 1; }
  tail -2 gpurun_out/tune_v910_$WL.log
done
ms() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['ms_per_step'],3))" $1; }
for r in 1 2; do
  for WL in cond-unet dit; do
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 30 --workload $WL > gpurun_out/v910_base_$WL$r.log 2>&1 || exit 1
    SDMI_TUNED_GEMM=gpurun_out/tuned_v910.json timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 30 --workload $WL > gpurun_out/v910_new_$WL$r.log 2>&1 || exit 1
    echo "$WL r$r base $(ms gpurun_out/v910_base_$WL$r.log) new $(ms gpurun_out/v910_new_$WL$r.log)"
  done
done
