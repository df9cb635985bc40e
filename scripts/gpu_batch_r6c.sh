#!/bin/bash
# round-6 batch: device-true timeline of the cond-UNet step (critical path, main-stream idle gaps), then the VQVAE
# workloads' profiles (kernel trace, PMC traffic, dominant-kernel roofline evidence)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
GAPS=40 TAG=r06a WL=cond-unet bash scripts/gpu_timeline.sh || exit 1
for W in vqvae vqvae-train; do TAG=r06 WL=$W bash scripts/gpu_profile.sh || exit 1; done
