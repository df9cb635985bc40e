#!/bin/bash
# Same-box A/B of env settings on the working tree: the bench alternating arms (ARMS: ';'-separated env strings,
# '.' = none), two rounds, per workload (WLS); optional GPU tests first (TESTS)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_envab.log 2>&1
  rc=$?; tail -2 gpurun_out/t_envab.log; [ $rc -eq 0 ] || exit 1
fi
ms() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['ms_per_step'],3))" $1; }
IFS=';' read -ra A <<< "${ARMS:-.}"
for W in ${WLS:-cond-unet}; do
  for r in 1 2; do
    i=0
    for E in "${A[@]}"; do
      i=$((i+1))
      if [ "$E" = "." ]; then EE=""; else EE="$E"; fi
      env $EE timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 30 $BARGS --workload $W > gpurun_out/envab_${W}_$i$r.log 2>&1 || { tail -5 gpurun_out/envab_${W}_$i$r.log; exit 1; }
      echo "$W [$E] r$r $(ms gpurun_out/envab_${W}_$i$r.log)"
    done
  done
done
