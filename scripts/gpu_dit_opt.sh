#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_dit_gpu.py tests/test_plan_gpu.py tests/test_dp_gpu.py tests/test_leaf_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_ditopt.log 2>&1 || { tail -30 gpurun_out/t_ditopt.log; exit 1; }
tail -2 gpurun_out/t_ditopt.log
WL=dit A="SDMI_OPT_CHUNKS=1" B="SDMI_X=0" TAG=dopt bash scripts/gpu_ab2.sh || exit 1
WL=dit A="SDMI_OPT_CHUNKS=3" B="SDMI_OPT_CHUNKS=12" TAG=dopt2 bash scripts/gpu_ab2.sh
