#!/bin/bash
# Kernel trace of captured sampling (one reverse step between two ddpm_prev_kernel launches): per-kernel time and the
# main stream's idle gaps (scripts/critical_path.py --marker ddpm_prev_kernel)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for SB in ${SBS:-1 8}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sp_$SB -o run -- python3 bench.py --no-cpu-baseline --workload sample --sample-batch $SB --steps 20 --warmup 3 > gpurun_out/sp_$SB.log 2>&1 || { tail -20 gpurun_out/sp_$SB.log; exit 1; }
  tail -1 gpurun_out/sp_$SB.log | cut -c1-160
  python scripts/critical_path.py gpurun_out/sp_$SB/run_kernel_trace.csv --marker ddpm_prev_kernel --gaps 30 > gpurun_out/cp_s$SB.txt
  head -40 gpurun_out/cp_s$SB.txt
done
