#!/bin/bash
# Persistent streaming GEMM (variants 12-15): numerics tests, per-shape tuning against the current table on the
# forward / data-gradient launches of the cond-UNet and DiT steps, then the steps with the re-tuned table vs the old.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
TAG=${TAG:-st}
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tst_$TAG.log 2>&1 || { tail -40 gpurun_out/tst_$TAG.log; exit 1; }
tail -1 gpurun_out/tst_$TAG.log
cp stablediffusion-pytorch_amd/sdmi/tuned_gemm.json gpurun_out/tuned_$TAG.json
for W in ${WLS:-dit cond-unet}; do
  SDMI_TUNE_VARIANTS=12,13,14,15 timeout -k 10 400 python -u scripts/tune_gemm.py --workload $W --against-table --skip-colmajor --out gpurun_out/tuned_$TAG.json > gpurun_out/tune_${TAG}_$W.log 2>&1 || { tail -20 gpurun_out/tune_${TAG}_$W.log; exit 1; }
  tail -2 gpurun_out/tune_${TAG}_$W.log
done
ms() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['ms_per_step'],3))" $1; }
for W in ${WLS:-dit cond-unet}; do
  for r in 1 2; do
    timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 30 --workload $W > gpurun_out/ab_${TAG}_${W}_old$r.log 2>&1 || { tail -5 gpurun_out/ab_${TAG}_${W}_old$r.log; exit 1; }
    SDMI_TUNED_GEMM=gpurun_out/tuned_$TAG.json timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 30 --workload $W > gpurun_out/ab_${TAG}_${W}_new$r.log 2>&1 || { tail -5 gpurun_out/ab_${TAG}_${W}_new$r.log; exit 1; }
    echo "$W run$r old $(ms gpurun_out/ab_${TAG}_${W}_old$r.log) new $(ms gpurun_out/ab_${TAG}_${W}_new$r.log) ms"
  done
done
