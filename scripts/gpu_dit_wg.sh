#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_dit_gpu.py tests/test_plan_gpu.py tests/test_dp_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_ditwg.log 2>&1 || { tail -30 gpurun_out/t_ditwg.log; exit 1; }
tail -2 gpurun_out/t_ditwg.log
WL=dit A="SDMI_DIT_WG_STREAMS=0" B="SDMI_DIT_WG_STREAMS=2" TAG=dwg bash scripts/gpu_ab2.sh || exit 1
WL=dit A="SDMI_DIT_WG_STREAMS=1" B="SDMI_DIT_WG_STREAMS=3" TAG=dwg2 bash scripts/gpu_ab2.sh
