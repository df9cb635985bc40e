cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for C in fwd wg1v2 wg6v2 wg3v11; do timeout -k 10 60 python3 scripts/conv_pmc_probe.py $C 2>&1 | grep -v amdgpu; SDMI_LIB_PATH=$GRAFT_REPO_ROOT/abprev/libsdmi.so timeout -k 10 60 python3 scripts/conv_pmc_probe.py $C 2>&1 | grep -v amdgpu | sed 's/^/old /'; done
TESTS="tests/test_gemm_reduce_gpu.py tests/test_gemm_gpu.py tests/test_unet_gpu.py tests/test_dit_gpu.py tests/test_vqvae_gpu.py tests/test_bench_step_gpu.py tests/test_mnist_gpu.py" WLS="cond-unet dit" bash scripts/gpu_ab_lib.sh
