#!/bin/bash
# GPU pass: the whole -m gpu suite (assertion failures do not stop the pass; a crash / timeout does), then the
# headline bench (plan replay) and the eager-issue bench for the host-issue comparison.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-t}
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -rf > gpurun_out/t_$TAG.log 2>&1
rc=$?
tail -30 gpurun_out/t_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/b_$TAG.log 2>&1 || { tail -20 gpurun_out/b_$TAG.log; exit 1; }
tail -1 gpurun_out/b_$TAG.log | cut -c1-400
timeout -k 10 300 python -u bench.py --no-cpu-baseline --issue eager > gpurun_out/be_$TAG.log 2>&1 || { tail -20 gpurun_out/be_$TAG.log; exit 1; }
tail -1 gpurun_out/be_$TAG.log | cut -c1-300
