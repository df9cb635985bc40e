#!/bin/bash
# GEMM table entries for the VQVAE training step (its launches ran on the built-in split heuristic, capped at 16
# splits: 16-144 workgroups for the 256^2 weight gradients), then a same-box A/B of the VQVAE lines with the new table.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
cp stablediffusion-pytorch_amd/sdmi/tuned_gemm.json gpurun_out/tuned_vq.json
timeout -k 10 900 python -u scripts/tune_gemm.py --workload vqvae-train --out gpurun_out/tuned_vq.json > gpurun_out/tune_vq.log 2>&1 || { tail -30 gpurun_out/tune_vq.log; exit 1; }
tail -3 gpurun_out/tune_vq.log
ARMS=".;SDMI_TUNED_GEMM=gpurun_out/tuned_vq.json" WLS="vqvae-train vqvae" BARGS="--steps 20" bash scripts/gpu_env_ab.sh
