#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/wg_anatomy.py > gpurun_out/wga.txt 2>&1 || { tail -20 gpurun_out/wga.txt; exit 1; }
cat gpurun_out/wga.txt
SPLITS=1,4 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_wga -o run -- python3 scripts/wg_anatomy.py > gpurun_out/wga_prof.log 2>&1 || { tail -20 gpurun_out/wga_prof.log; exit 1; }
head -30 gpurun_out/prof_wga/run_kernel_stats.csv | cut -c1-200
