#!/bin/bash
# same-box A/B of the working tree under env settings (scripts/gpu_bisect.sh arms)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
ARMS="${ARMS:-. .:SDMI_SIDE_PRIORITY=1 .:SDMI_SIDE_PRIORITY=2 .:SDMI_SIDE_PRIORITY=3}" bash scripts/gpu_bisect.sh
