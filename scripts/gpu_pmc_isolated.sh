#!/bin/bash
# HBM traffic per launch from PMC counters with every launch of one recorded cond-UNet step re-issued ALONE
# (scripts/plan_profile.py, PLAN_PROFILE_ITERS=0,1): separate rocprofv3 passes for FETCH_SIZE and WRITE_SIZE, each
# with --kernel-trace (grid z per dispatch); FETCH_SIZE x2 (gfx950 correction, MI355X_MICROARCH.md HBM section).
# The last quarter of each kernel's dispatches are the isolated re-issues (3 step executions precede them).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r04}
mkdir -p gpurun_out
for C in FETCH_SIZE WRITE_SIZE; do
  PLAN_PROFILE_ITERS=0,1 PLAN_PROFILE_NO_BLAS=1 timeout -s KILL 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/ipmc_${TAG}_$C -o run -- python3 scripts/plan_profile.py > gpurun_out/ipmc_${TAG}_$C.log 2>&1 || { tail -5 gpurun_out/ipmc_${TAG}_$C.log; exit 1; }
done
python3 scripts/pmc_summary.py gpurun_out/ipmc_${TAG}_FETCH_SIZE gpurun_out/ipmc_${TAG}_WRITE_SIZE --tail-frac 0.25 --json gpurun_out/${TAG}_pmc_traffic.json > gpurun_out/${TAG}_pmc_summary.txt
head -30 gpurun_out/${TAG}_pmc_summary.txt
python3 scripts/roofline_evidence.py gpurun_out/ipmc_${TAG}_FETCH_SIZE gpurun_out/ipmc_${TAG}_FETCH_SIZE gpurun_out/ipmc_${TAG}_WRITE_SIZE "${ROOF_KERNEL:-gemm_dma_kernel<1, 0, 2, 128>}" --tail-frac 0.25 --json gpurun_out/${TAG}_roofline_evidence.json
