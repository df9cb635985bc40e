#!/bin/bash
# isolated per-op profile of the recorded step + weight-gradient variant probe
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-pp}
PLAN_PROFILE_JSON=gpurun_out/pp_$TAG.json timeout -k 10 400 python -u scripts/plan_profile.py --top 90 > gpurun_out/pp_$TAG.txt 2>&1 || { tail -20 gpurun_out/pp_$TAG.txt; exit 1; }
head -40 gpurun_out/pp_$TAG.txt
for v in 0 2 3; do
  SDMI_GEMM_VARIANT=$v SPLITS=1,4,8,16,32 timeout -k 10 200 python -u scripts/wgrad_probe.py > gpurun_out/wg_${TAG}_$v.txt 2>&1 || { tail -20 gpurun_out/wg_${TAG}_$v.txt; exit 1; }
done
