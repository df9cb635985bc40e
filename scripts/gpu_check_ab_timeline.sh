cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_unet_gpu.py tests/test_bench_step_gpu.py -m gpu -x -q -k "groupnorm or full or bench_step" --timeout 200 --timeout-method thread > gpurun_out/t_o.log 2>&1
rc=$?; tail -2 gpurun_out/t_o.log; [ $rc -eq 0 ] || exit 1
ARMS="abprev ." bash scripts/gpu_bisect.sh || exit 1
TAG=r04c bash scripts/gpu_timeline.sh
