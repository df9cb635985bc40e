#!/bin/bash
# Round-2 verification on one GPU: parity suite, smoke(), headline bench (with the CPU baseline), secondary workloads,
# rocprofv3 kernel stats + trace summary, PMC HBM traffic of the roofline kernel (separate FETCH / WRITE passes).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-f2}
step() { echo "== $1"; }
step tests
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1 || { tail -40 gpurun_out/t_$TAG.log; exit 1; }
tail -1 gpurun_out/t_$TAG.log
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
step bench
timeout -k 10 400 python -u bench.py > gpurun_out/b_$TAG.log 2>&1 || { tail -20 gpurun_out/b_$TAG.log; exit 1; }
tail -1 gpurun_out/b_$TAG.log | cut -c1-300
for wl in dit uncond-unet vqvae vqvae-train sample; do
  step "bench $wl"
  timeout -k 10 400 python -u bench.py --workload $wl > gpurun_out/b_${TAG}_$wl.log 2>&1 || { tail -20 gpurun_out/b_${TAG}_$wl.log; exit 1; }
  tail -1 gpurun_out/b_${TAG}_$wl.log | cut -c1-200
done
step rocprof
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1 || { tail -20 gpurun_out/prof_$TAG.log; exit 1; }
python3 scripts/trace_summary.py gpurun_out/prof_$TAG/run_kernel_trace.csv --top 60 > gpurun_out/ts_$TAG.txt
head -8 gpurun_out/ts_$TAG.txt
step pmc
TAG=$TAG bash scripts/gpu_pmc.sh > gpurun_out/pmcrun_$TAG.log 2>&1 || { tail -20 gpurun_out/pmcrun_$TAG.log; exit 1; }
tail -5 gpurun_out/pmcrun_$TAG.log
