#!/bin/bash
# bench line + isolated per-op profile of the recorded step
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-bp}
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/b_$TAG.log 2>&1 || { tail -20 gpurun_out/b_$TAG.log; exit 1; }
tail -1 gpurun_out/b_$TAG.log | cut -c1-240
PLAN_PROFILE_JSON=gpurun_out/pp_$TAG.json timeout -k 10 400 python -u scripts/plan_profile.py --top 90 > gpurun_out/pp_$TAG.txt 2>&1 || { tail -20 gpurun_out/pp_$TAG.txt; exit 1; }
head -34 gpurun_out/pp_$TAG.txt | grep -v amdgpu.ids
