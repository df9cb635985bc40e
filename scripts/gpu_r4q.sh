cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
SDMI_LEAD_CHUNKS=1 TAG=r04d bash scripts/gpu_timeline.sh || exit 1
WL=dit TAG=r04dit bash scripts/gpu_profile.sh
