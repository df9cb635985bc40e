#!/bin/bash
# round-6 batch: in-launch combine A/B for the forward / data-gradient GEMMs (sampler B = 1, headline step), then the
# VQVAE workloads' profiles (kernel trace, PMC traffic, dominant-kernel roofline evidence)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
SUITE=0 WLS="sample cond-unet" MODES="0 dg" TAG=fix3 bash scripts/gpu_fix_ab.sh || exit 1
for W in vqvae vqvae-train; do TAG=r06 WL=$W bash scripts/gpu_profile.sh || exit 1; done
