#!/bin/bash
# DiT step across prebuilt trees ab_<rev>/ (package + bench.py) and the working tree, alternating, same box
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
ms() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['ms_per_step'],3))" $1; }
W=${AB_WORKLOAD:-dit}
for r in 1 2; do
  for d in ${AB_DIRS}; do
    rm -rf /tmp/abx && mkdir -p /tmp/abx && cp -r $d/stablediffusion-pytorch_amd $d/bench.py /tmp/abx/ && cp -r tests oracle profiles /tmp/abx/
    (cd /tmp/abx && timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 30 --workload $W > $GRAFT_REPO_ROOT/gpurun_out/bis.log 2>&1) || { tail -5 gpurun_out/bis.log; exit 1; }
    echo "$d $(ms gpurun_out/bis.log)"
  done
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 30 --workload $W > gpurun_out/bis.log 2>&1 || { tail -5 gpurun_out/bis.log; exit 1; }
  echo "new $(ms gpurun_out/bis.log)"
done
