#!/bin/bash
# Same-box headline bench over several trees (ab_* copies of earlier commits with their prebuilt libraries) and env
# settings of the working tree, alternating, two rounds: ARMS="dir[:ENV=V,...] ..." (dir "." = working tree);
# BENCH_ARGS: extra bench.py arguments (e.g. "--workload dit")
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
ms() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['ms_per_step'],3))" $1; }
i=0
for A in $ARMS; do
  d=${A%%:*}; e=""; [ "$A" != "$d" ] && e=${A#*:}
  if [ "$d" != "." ]; then
    rm -rf /tmp/arm$i && mkdir -p /tmp/arm$i && cp -r $d/stablediffusion-pytorch_amd $d/bench.py /tmp/arm$i/ && cp -r tests oracle profiles /tmp/arm$i/
  fi
  i=$((i+1))
done
for r in 1 2; do
  i=0
  for A in $ARMS; do
    d=${A%%:*}; e=""; [ "$A" != "$d" ] && e=${A#*:}
    wd=$GRAFT_REPO_ROOT; [ "$d" != "." ] && wd=/tmp/arm$i
    (cd $wd && env ${e//,/ } timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 30 $BENCH_ARGS > $GRAFT_REPO_ROOT/gpurun_out/bis_${i}_${r}.log 2>&1) || { tail -5 gpurun_out/bis_${i}_${r}.log; exit 1; }
    echo "$A r$r $(ms gpurun_out/bis_${i}_${r}.log)"
    i=$((i+1))
  done
done
