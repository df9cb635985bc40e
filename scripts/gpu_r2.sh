#!/bin/bash
# round-2 GPU pass: full -m gpu suite, headline bench, sampling bench
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r2}
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -rf > gpurun_out/t_$TAG.log 2>&1
rc=$?
grep -E "passed|failed" gpurun_out/t_$TAG.log | tail -3; grep -E "^FAILED" gpurun_out/t_$TAG.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/b_$TAG.log 2>&1 || { tail -20 gpurun_out/b_$TAG.log; exit 1; }
tail -1 gpurun_out/b_$TAG.log | cut -c1-250
timeout -k 10 300 python -u bench.py --workload sample --steps 50 --warmup 3 > gpurun_out/bs_$TAG.log 2>&1 || { tail -20 gpurun_out/bs_$TAG.log; exit 1; }
tail -1 gpurun_out/bs_$TAG.log | cut -c1-900
