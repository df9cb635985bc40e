#!/bin/bash
# Re-tune the split-K / mainloop table of one workload on the GPU (table written under gpurun_out/).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
WL=${WL:-cond-unet}
timeout -k 10 1000 python -u scripts/tune_gemm.py --workload $WL --out gpurun_out/tuned_$WL.json > gpurun_out/tune_$WL.log 2>&1 || { tail -20 gpurun_out/tune_$WL.log; exit 1; }
tail -3 gpurun_out/tune_$WL.log
