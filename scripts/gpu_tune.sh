#!/bin/bash
# re-tune the split-K / mainloop table on the step's GEMMs, then bench with it
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-tune}
WL=${WL:-cond-unet}
cp stablediffusion-pytorch_amd/sdmi/tuned_gemm.json gpurun_out/tuned_gemm.json
timeout -k 10 900 python -u scripts/tune_gemm.py --workload $WL --out gpurun_out/tuned_gemm.json > gpurun_out/tune_$TAG.log 2>&1 || { tail -20 gpurun_out/tune_$TAG.log; exit 1; }
tail -3 gpurun_out/tune_$TAG.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/b0_$TAG.log 2>&1 && tail -1 gpurun_out/b0_$TAG.log | cut -c1-200; SDMI_TUNED_GEMM=gpurun_out/tuned_gemm.json timeout -k 10 300 python -u bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/b_$TAG.log 2>&1 || { tail -20 gpurun_out/b_$TAG.log; exit 1; }
tail -1 gpurun_out/b_$TAG.log | cut -c1-240
