#!/bin/bash
# In-launch split-K combine (csrc/gemm.hip fixup_combine): its bitwise tests first, then the parity suite, then a
# same-box A/B of the headline and DiT steps with the combine off (SDMI_SPLITK_FIX=0: slabs + reducer launches) and on.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
TAG=${TAG:-fix}
timeout -k 10 300 python -u -m pytest tests/test_gemm_reduce_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tfix_$TAG.log 2>&1 || { tail -40 gpurun_out/tfix_$TAG.log; exit 1; }
tail -1 gpurun_out/tfix_$TAG.log
if [ "${SUITE:-1}" = 1 ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1 || { tail -40 gpurun_out/t_$TAG.log; exit 1; }
  tail -1 gpurun_out/t_$TAG.log
fi
ms() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['ms_per_step'],3))" $1; }
# MODES: SDMI_SPLITK_FIX values to compare (0 = reducer launches, wg / dg / 1 = in-launch combine for weight gradients /
# forward and data gradients / both); sample = the captured B = 1 DDPM loop (single stream)
for W in ${WLS:-cond-unet dit}; do
  EXTRA="--steps 30"
  [ "$W" = sample ] && EXTRA="--steps 100 --warmup 10"
  for r in 1 2; do
    for F in ${MODES:-0 1}; do
      SDMI_SPLITK_FIX=$F timeout -k 10 200 python -u bench.py --no-cpu-baseline $EXTRA --workload $W > gpurun_out/ab_${TAG}_${W}_f$F$r.log 2>&1 || { tail -5 gpurun_out/ab_${TAG}_${W}_f$F$r.log; exit 1; }
      echo "$W fix=$F run$r $(ms gpurun_out/ab_${TAG}_${W}_f$F$r.log) ms"
    done
  done
done
