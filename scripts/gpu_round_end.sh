#!/bin/bash
# Round-end evidence in one call: parity suite + smoke + default bench + kernel trace (gpu_final.sh), the secondary
# bench lines (gpu_secondary.sh) and the headline profile with PMC traffic and roofline evidence (gpu_profile.sh)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
T=${TAG:-r04f}
TAG=$T bash scripts/gpu_final.sh || exit 1
TAG=$T bash scripts/gpu_secondary.sh || exit 1
TAG=$T bash scripts/gpu_profile.sh || exit 1
