#!/bin/bash
# Streams vs hardware queues: the plain step with the gradient-norm pieces on their own stream vs on the engine's
# context stream (idle in the backward), the forced-reducer step (RCCL group of one) likewise for the reducer stream,
# then a kernel trace of the forced-reducer step for scripts/critical_path.py
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
ARMS=".;SDMI_NORM_STREAM=ctx" bash scripts/gpu_env_ab.sh || exit 1
BARGS=--force-reducer ARMS=".;SDMI_RED_STREAM=ctx" bash scripts/gpu_env_ab.sh || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/frt -o run -- python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline --force-reducer > gpurun_out/frt.log 2>&1 || { tail -20 gpurun_out/frt.log; exit 1; }
f=$(ls gpurun_out/frt/*/run_kernel_trace.csv gpurun_out/frt/run_kernel_trace.csv 2>/dev/null | tail -1)
python3 scripts/critical_path.py $f > gpurun_out/cp_frt.txt && head -12 gpurun_out/cp_frt.txt
