cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_bench_step_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_g1.log 2>&1
rc=$?; tail -2 gpurun_out/t_g1.log; [ $rc -eq 0 ] || exit 1
ARMS="ab_old ." bash scripts/gpu_bisect.sh
