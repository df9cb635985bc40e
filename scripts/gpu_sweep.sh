#!/bin/bash
# Same-box sweep of env configurations of the headline bench: CFGS="cfgA;cfgB;..." (each a space-separated env list,
# "-" = defaults), REPS rounds in alternation.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
IFS=';' read -ra C <<< "$CFGS"
for i in $(seq 1 ${REPS:-2}); do
  for cfg in "${C[@]}"; do
    e=$cfg; [ "$e" = "-" ] && e=""
    env $e timeout -k 10 300 python -u bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/b_sweep.log 2>&1 || { tail -20 gpurun_out/b_sweep.log; exit 1; }
    python3 -c "import json;d=json.loads(open('gpurun_out/b_sweep.log').read().strip().splitlines()[-1]);print('$cfg', round(d['ms_per_step'],3), d.get('last_loss'))"
  done
done
