#!/bin/bash
# VQ kernels check: the VQVAE / latent / leaf parity tests, then the two VQVAE bench lines.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_vqvae_gpu.py tests/test_vqvae_train_gpu.py tests/test_latent_gen_gpu.py tests/test_leaf_gpu.py tests/test_leafops_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_vq.log 2>&1 || { tail -40 gpurun_out/t_vq.log; exit 1; }
tail -1 gpurun_out/t_vq.log
for W in vqvae vqvae-train; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --workload $W --steps 20 > gpurun_out/bvq_$W.log 2>&1 || { tail -5 gpurun_out/bvq_$W.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],3))" gpurun_out/bvq_$W.log $W
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_vq -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --workload vqvae-train > gpurun_out/prof_vq.log 2>&1 || { tail -5 gpurun_out/prof_vq.log; exit 1; }
grep -E "vq_" gpurun_out/prof_vq/run_kernel_stats.csv | cut -c1-160
