#!/bin/bash
# Same-box env-knob A/B of the headline step: the tree as is vs each ENVS entry (space-separated VAR=VALUE lists,
# ';'-separated arms), alternating, ROUNDS rounds
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
ms() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['ms_per_step'],3))" $1; }
W=${AB_WORKLOAD:-cond-unet}
IFS=';' read -ra ARMS <<< "$ENVS"
for r in $(seq 1 ${ROUNDS:-2}); do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 30 --workload $W > gpurun_out/ea.log 2>&1 || { tail -5 gpurun_out/ea.log; exit 1; }
  echo "base $r $(ms gpurun_out/ea.log)"
  for E in "${ARMS[@]}"; do
    env $E timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 30 --workload $W > gpurun_out/ea.log 2>&1 || { tail -5 gpurun_out/ea.log; exit 1; }
    echo "$E $r $(ms gpurun_out/ea.log)"
  done
done
