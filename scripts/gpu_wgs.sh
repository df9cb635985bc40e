#!/bin/bash
# weight-gradient side streams: plan / DP / UNet parity with 2 streams, then bench A/B over the stream count
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
SDMI_WG_STREAMS=2 timeout -k 10 600 python -u -m pytest tests/test_plan_gpu.py tests/test_dp_gpu.py tests/test_unet_gpu.py tests/test_rccl_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_wgs.log 2>&1 || { tail -30 gpurun_out/t_wgs.log; exit 1; }
tail -2 gpurun_out/t_wgs.log
A="SDMI_WG_STREAMS=1" B="SDMI_WG_STREAMS=2" TAG=wgs2 bash scripts/gpu_ab2.sh
A="SDMI_WG_STREAMS=3" B="SDMI_WG_STREAMS=4" TAG=wgs3 bash scripts/gpu_ab2.sh
