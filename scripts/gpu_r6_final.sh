#!/bin/bash
# Round-6 closing run, part 1 on one GPU: parity suite + smoke + default bench + kernel trace (gpu_final.sh), then the
# CU-masked queue probe once under rocprofv3 after its teardown fix (round-5 verdict weak #7).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
TAG=${TAG:-r06f}
TAG=$TAG bash scripts/gpu_final.sh || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/qp_cumask_$TAG -o run -- python3 scripts/queue_probe.py cumask > gpurun_out/qp_cumask_$TAG.log 2>&1
rc=$?
echo "queue_probe cumask exit $rc"; tail -4 gpurun_out/qp_cumask_$TAG.log
exit $rc
