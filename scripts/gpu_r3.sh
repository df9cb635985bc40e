#!/bin/bash
# Round-3 GPU check: the parity suite (incl. the new B=32 plan-step, GradScaler, C-ABI, DDIM tests), smoke(), the
# headline bench and the sampling line. TAG names the outputs under gpurun_out/.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r3}
mkdir -p gpurun_out
step() { echo "== $1 $(date +%T)"; }
step tests
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread ${TESTS:-} > gpurun_out/t_$TAG.log 2>&1
rc=$?
tail -30 gpurun_out/t_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi   # 1 = test failures (report them, keep going); else stop
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
step bench
timeout -k 10 400 python -u bench.py > gpurun_out/b_$TAG.log 2>&1 || { tail -20 gpurun_out/b_$TAG.log; exit 1; }
tail -1 gpurun_out/b_$TAG.log | cut -c1-400
exit $rc
