#!/bin/bash
# Same-box A/B of two libraries under the SAME Python tree: abprev/libsdmi.so (a previous build) vs the tree's, the
# bench alternating old / new per workload (WLS, default cond-unet), two rounds; optional GPU tests first (TESTS) and
# extra env arms on the new library (ENV1 / ENV2, e.g. ENV1="SDMI_TUNED_GEMM=gpurun_out/t.json").
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_ablib.log 2>&1
  rc=$?; tail -2 gpurun_out/t_ablib.log; [ $rc -eq 0 ] || exit 1
fi
ms() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['ms_per_step'],3))" $1; }
OLD=$GRAFT_REPO_ROOT/abprev/libsdmi.so
for W in ${WLS:-cond-unet}; do
  for r in 1 2; do
    if [ -e "$OLD" ]; then
      SDMI_LIB_PATH=$OLD timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 30 --workload $W > gpurun_out/ablib_old_$W$r.log 2>&1 || { tail -5 gpurun_out/ablib_old_$W$r.log; exit 1; }
      echo "$W old$r $(ms gpurun_out/ablib_old_$W$r.log)"
    fi
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 30 --workload $W > gpurun_out/ablib_new_$W$r.log 2>&1 || { tail -5 gpurun_out/ablib_new_$W$r.log; exit 1; }
    echo "$W new$r $(ms gpurun_out/ablib_new_$W$r.log)"
    for E in "$ENV1" "$ENV2"; do
      [ -n "$E" ] || continue
      env $E timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 30 --workload $W > gpurun_out/ablib_env_$W$r.log 2>&1 || { tail -5 gpurun_out/ablib_env_$W$r.log; exit 1; }
      echo "$W new+$E $r $(ms gpurun_out/ablib_env_$W$r.log)"
    done
  done
done
