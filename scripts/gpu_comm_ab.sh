#!/bin/bash
# Native RCCL bucket all-reduce (csrc/comm.hip) vs torch.distributed callouts: the RCCL / data-parallel GPU tests,
# then the forced-reducer and plain step A/B with the stream -> hardware-queue map of each arm
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_rccl_gpu.py tests/test_dp_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t_comm.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/t_comm.log | tail -12; [ $rc -eq 0 ] || exit 1
ARMS="${ARMS:-SDMI_NATIVE_COMM=0;.}" bash scripts/gpu_queue_ab.sh
