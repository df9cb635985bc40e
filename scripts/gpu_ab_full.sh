#!/bin/bash
# Same-box A/B of the whole tree (python + libsdmi.so) against the copy in abprev/ (a previous commit's package and
# bench.py, library prebuilt): the GPU suite first, then the headline bench alternating old / new; AB_ENV_NEW adds env
# settings to extra "new" arms, e.g. AB_ENV_NEW="SDMI_GRAD_WIRE=bf16".
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
if [ "${AB_TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_ab.log 2>&1
  rc=$?; tail -3 gpurun_out/t_ab.log; [ $rc -eq 0 ] || exit 1
fi
rm -rf /tmp/abold && mkdir -p /tmp/abold && cp -r abprev/stablediffusion-pytorch_amd abprev/bench.py /tmp/abold/ && cp -r tests oracle profiles /tmp/abold/
ms() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['ms_per_step'],3))" $1; }
W=${AB_WORKLOAD:-cond-unet}
for r in 1 2; do
  (cd /tmp/abold && timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 30 --workload $W > $GRAFT_REPO_ROOT/gpurun_out/ab_old$r.log 2>&1) || { tail -5 gpurun_out/ab_old$r.log; exit 1; }
  echo "old$r $(ms gpurun_out/ab_old$r.log)"
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 30 --workload $W > gpurun_out/ab_new$r.log 2>&1 || { tail -5 gpurun_out/ab_new$r.log; exit 1; }
  echo "new$r $(ms gpurun_out/ab_new$r.log)"
  for E in "$AB_ENV_NEW" "$AB_ENV_NEW2" "$AB_ENV_NEW3"; do
    [ -n "$E" ] || continue
    env $E timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 30 --workload $W > gpurun_out/ab_env$r.log 2>&1 || { tail -5 gpurun_out/ab_env$r.log; exit 1; }
    echo "new+$E $r $(ms gpurun_out/ab_env$r.log)"
  done
done
if [ -n "$AB_ATTN" ]; then
  timeout -k 10 300 python -u scripts/attn_bench.py > gpurun_out/attn_new.txt 2>&1 && cat gpurun_out/attn_new.txt
fi
