#!/bin/bash
# Round-3 A/B: optional GPU tests (TESTS="file::name ..."), then the headline bench with env A vs env B on the same box,
# alternated REPS times. Usage: TESTS=... A="SDMI_X=0" B="SDMI_X=1" REPS=2 bash scripts/gpu_ab3.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-ab3}
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -q -x --timeout 300 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1
  rc=$?; tail -5 gpurun_out/t_$TAG.log
  [ $rc -ne 0 ] && exit $rc
fi
for i in $(seq 1 ${REPS:-2}); do
  for arm in A B; do
    envs=${!arm}
    env $envs timeout -k 10 300 python -u bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/b_${TAG}_$arm$i.log 2>&1 || { tail -20 gpurun_out/b_${TAG}_$arm$i.log; exit 1; }
    python3 -c "import json,sys;d=json.loads(open('gpurun_out/b_${TAG}_$arm$i.log').read().strip().splitlines()[-1]);print('$arm', '$envs', round(d['ms_per_step'],3), d.get('last_loss'))"
  done
done
