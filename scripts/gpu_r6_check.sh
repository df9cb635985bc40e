#!/bin/bash
# Round-6 check on one GPU: the parity suite (incl. the DDP-caller and staged-backward tests), the CU-masked queue probe
# once after its teardown fix (round-5 verdict: SIGSEGV in __cxa_finalize), then the VQVAE workloads' profiles
# (gpu_profile.sh: kernel trace, PMC traffic, dominant-kernel roofline evidence).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
TAG=${TAG:-r06a}
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1 || { tail -40 gpurun_out/t_$TAG.log; exit 1; }
tail -1 gpurun_out/t_$TAG.log
if [ "${PROBE:-1}" = 1 ]; then
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/qp_cumask_$TAG -o run -- python3 scripts/queue_probe.py cumask > gpurun_out/qp_cumask_$TAG.log 2>&1 || { echo "queue_probe cumask FAILED: $?"; tail -5 gpurun_out/qp_cumask_$TAG.log; exit 1; }
  echo "queue_probe cumask exit 0"; tail -3 gpurun_out/qp_cumask_$TAG.log
fi
for W in ${WLS:-vqvae vqvae-train}; do TAG=$TAG WL=$W bash scripts/gpu_profile.sh || exit 1; done
