#!/bin/bash
# step time vs per-GPU batch (how much of the step is latency-bound): cond-UNet and DiT at B = 8, 16, 32
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
ms() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['ms_per_step'],3))" $1; }
for W in cond-unet dit; do
  for B in 8 16 32; do
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 20 --batch $B --workload $W > gpurun_out/bs_${W}_$B.log 2>&1 || { tail -5 gpurun_out/bs_${W}_$B.log; exit 1; }
    echo "$W B=$B $(ms gpurun_out/bs_${W}_$B.log)"
  done
done
