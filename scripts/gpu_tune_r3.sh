#!/bin/bash
# Re-tune the per-shape GEMM table over every mainloop variant (incl. the round-3 deep rings 6 / 7 / 8), then bench the
# headline step with the old and the new table on the same box (A/B).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-tune3}
mkdir -p gpurun_out
echo "== tune $(date +%T)"
timeout -k 10 900 python -u scripts/tune_gemm.py --out gpurun_out/tuned_$TAG.json > gpurun_out/tune_$TAG.log 2>&1 || { tail -20 gpurun_out/tune_$TAG.log; exit 1; }
tail -3 gpurun_out/tune_$TAG.log
for i in 1 2; do
  echo "== bench old table $(date +%T)"
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/b_${TAG}_old$i.log 2>&1 || { tail -20 gpurun_out/b_${TAG}_old$i.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/b_${TAG}_old$i.log').read().strip().splitlines()[-1]);print('old',d['ms_per_step'])"
  echo "== bench new table $(date +%T)"
  SDMI_TUNED_GEMM=gpurun_out/tuned_$TAG.json timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/b_${TAG}_new$i.log 2>&1 || { tail -20 gpurun_out/b_${TAG}_new$i.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/b_${TAG}_new$i.log').read().strip().splitlines()[-1]);print('new',d['ms_per_step'])"
done
