#!/bin/bash
# rocprofv3 kernel traces of the headline bench for the tree in abprev/ and the working tree (same box), each summarised
# by scripts/trace_summary.py; TRACE_ENV_NEW adds env settings to the working-tree run.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -rf /tmp/abold && mkdir -p /tmp/abold && cp -r abprev/stablediffusion-pytorch_amd abprev/bench.py /tmp/abold/ && cp -r tests oracle profiles /tmp/abold/
(cd /tmp/abold && timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/tr_old -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/tr_old.log 2>&1) || { tail -5 gpurun_out/tr_old.log; exit 1; }
python3 scripts/trace_summary.py gpurun_out/tr_old/run_kernel_trace.csv --top 100 > gpurun_out/ts_old.txt
head -8 gpurun_out/ts_old.txt
env $TRACE_ENV_NEW timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr_new -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/tr_new.log 2>&1 || { tail -5 gpurun_out/tr_new.log; exit 1; }
python3 scripts/trace_summary.py gpurun_out/tr_new/run_kernel_trace.csv --top 100 > gpurun_out/ts_new.txt
head -8 gpurun_out/ts_new.txt
