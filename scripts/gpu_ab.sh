#!/bin/bash
# A/B of step-level knobs: one bench line per configuration (env assignments in $CONFIGS, ';'-separated)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-ab}
IFS=';' read -ra CFG <<< "${CONFIGS:-BASE=1}"
i=0
for c in "${CFG[@]}"; do
  env $c timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/ab_${TAG}_$i.log 2>&1 || { echo "[$c] failed"; tail -5 gpurun_out/ab_${TAG}_$i.log; exit 1; }
  echo "[$c] $(tail -1 gpurun_out/ab_${TAG}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "ms")')"
  i=$((i+1))
done
