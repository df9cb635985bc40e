#!/bin/bash
# Sampling step: in-launch split-K combine (SDMI_SPLITK_FUSED) vs the reducer launch, B = 1 / 8, alternating
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
ms() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['ms_per_step'],3))" $1; }
for B in 1 8; do
  for r in 1 2; do
    for F in 0 2 4 16 64; do
      SDMI_SPLITK_FUSED=$F timeout -k 10 200 python -u bench.py --workload sample --sample-batch $B --steps 40 --no-cpu-baseline > gpurun_out/g.log 2>&1 || { tail -20 gpurun_out/g.log; exit 1; }
      echo "B=$B fused<=$F $(ms gpurun_out/g.log)"
    done
  done
done
