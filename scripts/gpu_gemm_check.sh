#!/bin/bash
# GEMM variant check: numerics for each mainloop variant, then the shape micro-benchmark.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in ${VARIANTS:-2}; do
  SDMI_GEMM_VARIANT=$v timeout -k 10 300 python -m pytest tests/test_gemm_gpu.py -x -q > gpurun_out/gemm_test_v$v.log 2>&1 || { tail -30 gpurun_out/gemm_test_v$v.log; exit 1; }
  tail -1 gpurun_out/gemm_test_v$v.log
done
for v in ${BENCH_VARIANTS:-0 2}; do
  SDMI_GEMM_VARIANT=$v timeout -k 10 120 python scripts/gemm_bench.py
done
