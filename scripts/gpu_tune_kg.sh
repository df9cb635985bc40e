#!/bin/bash
# The k-group weight-gradient mainloop (variant 11) tried against the current table's entry of every col-major (weight
# gradient) GEMM of the cond-UNet and DiT steps, then the headline and DiT bench with the updated table vs the package's
# table (same box, alternating), and the grouped weight-gradient launches on variant 11 as an env arm.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
T=${TAG:-kg}
cp stablediffusion-pytorch_amd/sdmi/tuned_gemm.json gpurun_out/tuned_$T.json
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_$T.log 2>&1
  rc=$?; tail -2 gpurun_out/t_$T.log; [ $rc -eq 0 ] || exit 1
fi
for WL in ${WLS:-cond-unet dit}; do
  SDMI_TUNE_VARIANTS=${VARS:-11} timeout -k 10 900 python -u scripts/tune_gemm.py --workload $WL --against-table ${MODESEL:---only-colmajor} --out gpurun_out/tuned_$T.json > gpurun_out/tune_${T}_$WL.log 2>&1 || { tail -5 gpurun_out/tune_${T}_$WL.log; exit 1; }
  tail -2 gpurun_out/tune_${T}_$WL.log
done
ms() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['ms_per_step'],3))" $1; }
for r in 1 2; do
  for WL in ${WLS:-cond-unet dit}; do
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 30 --workload $WL > gpurun_out/${T}_base_$WL$r.log 2>&1 || exit 1
    SDMI_TUNED_GEMM=gpurun_out/tuned_$T.json timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 30 --workload $WL > gpurun_out/${T}_new_$WL$r.log 2>&1 || exit 1
    SDMI_GROUPED_VARIANT=11 SDMI_TUNED_GEMM=gpurun_out/tuned_$T.json timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 30 --workload $WL > gpurun_out/${T}_grp_$WL$r.log 2>&1 || exit 1
    echo "$WL r$r base $(ms gpurun_out/${T}_base_$WL$r.log) new $(ms gpurun_out/${T}_new_$WL$r.log) new+grouped11 $(ms gpurun_out/${T}_grp_$WL$r.log)"
  done
done
