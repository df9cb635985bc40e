#!/bin/bash
# Round-end evidence (run as separate gpurun calls, each within its limit): PART=final -> parity suite + smoke + default
# bench + kernel trace (gpu_final.sh); PART=secondary -> the secondary bench lines (gpu_secondary.sh); PART=profile ->
# per-workload plan profile, trace, PMC traffic and roofline evidence of the bench kernel (gpu_profile.sh, WLS)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
T=${TAG:-r05}
case "${PART:-final}" in
  final) TAG=$T bash scripts/gpu_final.sh ;;
  secondary) TAG=$T bash scripts/gpu_secondary.sh ;;
  profile) for W in ${WLS:-cond-unet}; do TAG=$T WL=$W bash scripts/gpu_profile.sh || exit 1; done ;;
esac
