#!/bin/bash
# A/B of the headline bench: default tree vs environment overrides given as "A" / "B" (alternating, 2 rounds).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-ab}
for r in 1 2; do
  for arm in A B; do
    envs=${!arm}
    env $envs timeout -k 10 300 python -u bench.py --workload ${WL:-cond-unet} --no-cpu-baseline --steps 30 > gpurun_out/ab_${TAG}_${arm}$r.log 2>&1 || { tail -20 gpurun_out/ab_${TAG}_${arm}$r.log; exit 1; }
    echo "$arm$r [$envs] $(tail -1 gpurun_out/ab_${TAG}_${arm}$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "ms/step")')"
  done
done
