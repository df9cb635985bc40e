#!/bin/bash
# Sampling step with the inline context branch (inference): bench lines at B = 1 / 8 (DDPM) and DDIM B = 1, then a
# rocprofv3 kernel trace of the B = 1 DDPM sampling bench (per-kernel time of one reverse step, busy vs span)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_sampling_gpu.py -q --timeout 200 --timeout-method thread > gpurun_out/t_r3f.log 2>&1 || { tail -20 gpurun_out/t_r3f.log; exit 1; }
tail -1 gpurun_out/t_r3f.log
for B in 1 8; do
  timeout -k 10 300 python -u bench.py --workload sample --sample-batch $B --no-cpu-baseline > gpurun_out/bs${B}_r3f.log 2>&1 || { tail -20 gpurun_out/bs${B}_r3f.log; exit 1; }
  tail -1 gpurun_out/bs${B}_r3f.log | cut -c1-200
done
timeout -k 10 300 python -u bench.py --workload sample --sampler ddim --steps 50 --no-cpu-baseline > gpurun_out/bsd_r3f.log 2>&1 || { tail -20 gpurun_out/bsd_r3f.log; exit 1; }
tail -1 gpurun_out/bsd_r3f.log | cut -c1-200
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_s1 -o run -- python3 bench.py --workload sample --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_s1.log 2>&1 || { tail -20 gpurun_out/prof_s1.log; exit 1; }
python scripts/trace_summary.py gpurun_out/prof_s1/run_kernel_trace.csv --marker ddpm_prev_kernel --top 60 > gpurun_out/ts_s1.txt
head -40 gpurun_out/ts_s1.txt
