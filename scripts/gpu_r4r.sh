cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
SDMI_LEAD_CHUNKS=1 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_r.log 2>&1
rc=$?; tail -2 gpurun_out/t_r.log; [ $rc -eq 0 ] || exit 1
ARMS="ab_old . .:SDMI_LEAD_CHUNKS=1" bash scripts/gpu_bisect.sh || exit 1
SDMI_LEAD_CHUNKS=1 TAG=r04e bash scripts/gpu_timeline.sh
