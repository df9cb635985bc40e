#!/bin/bash
# the round's same-box gain: the round-2 final tree (ab_old/) against the working tree, cond-UNet and DiT-12L steps
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
AB_TESTS=0 bash scripts/gpu_ab_full.sh && AB_TESTS=0 AB_WORKLOAD=dit AB_ENV_NEW="SDMI_DIT_WG_GROUP=12" AB_ENV_NEW2="SDMI_NORM_PARTS=0" bash scripts/gpu_ab_full.sh
