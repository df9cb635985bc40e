#!/bin/bash
# Closing profile of the headline step on the current tree: isolated per-op plan profile, rocprofv3 kernel
# trace + stats, PMC HBM traffic (separate FETCH_SIZE / WRITE_SIZE passes), roofline evidence of the bench kernel
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-prof}
WL=${WL:-cond-unet}
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --no-cpu-baseline --workload $WL > gpurun_out/bench_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log | cut -c1-200
PLAN_PROFILE_JSON=gpurun_out/pp_$TAG.json timeout -k 10 400 python -u scripts/plan_profile.py --workload $WL --top 120 > gpurun_out/pp_$TAG.txt 2>&1 || { tail -20 gpurun_out/pp_$TAG.txt; exit 1; }
head -3 gpurun_out/pp_$TAG.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --workload $WL > gpurun_out/prof_$TAG.log 2>&1 || { tail -20 gpurun_out/prof_$TAG.log; exit 1; }
python scripts/trace_summary.py gpurun_out/prof_$TAG/run_kernel_trace.csv --top 80 > gpurun_out/ts_$TAG.txt
head -8 gpurun_out/ts_$TAG.txt
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/pmc_${TAG}_$C -o run -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --issue eager --workload $WL > gpurun_out/pmc_${TAG}_$C.log 2>&1 || { tail -5 gpurun_out/pmc_${TAG}_$C.log; exit 1; }
done
python3 scripts/pmc_summary.py gpurun_out/pmc_${TAG}_FETCH_SIZE gpurun_out/pmc_${TAG}_WRITE_SIZE --json gpurun_out/pmc_${TAG}_traffic.json > gpurun_out/pmc_${TAG}.txt
head -12 gpurun_out/pmc_${TAG}.txt
python3 scripts/roofline_evidence.py gpurun_out/prof_$TAG gpurun_out/pmc_${TAG}_FETCH_SIZE gpurun_out/pmc_${TAG}_WRITE_SIZE "${ROOF_KERNEL:-gemm_dma_kernel<1, 0, 2, 128>}" --json gpurun_out/${TAG}_roofline_evidence.json
cat gpurun_out/${TAG}_roofline_evidence.json
