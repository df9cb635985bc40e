#!/bin/bash
# kernel trace of the plan-replayed bench + host issue time + weight-gradient mainloop variants
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-p}
timeout -k 10 300 python -u -m pytest tests/test_unet_gpu.py::test_cond_trainer_two_steps_match_reference tests/test_mnist_gpu.py -q --timeout 200 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1
tail -3 gpurun_out/t_$TAG.log
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr_$TAG -o run -- python3 bench.py --steps 4 --warmup 3 --no-cpu-baseline > gpurun_out/tr_$TAG.log 2>&1 || { tail -20 gpurun_out/tr_$TAG.log; exit 1; }
python scripts/trace_summary.py gpurun_out/tr_$TAG/run_kernel_trace.csv --top 60 > gpurun_out/ts_$TAG.txt
head -8 gpurun_out/ts_$TAG.txt
timeout -k 10 200 python -u scripts/issue_time.py > gpurun_out/it_$TAG.log 2>&1; tail -3 gpurun_out/it_$TAG.log
for v in 0 2 3; do SPLITS=1,4,8,16 SDMI_GEMM_VARIANT=$v timeout -k 10 200 python -u scripts/wgrad_probe.py > gpurun_out/wg_${TAG}_$v.log 2>&1; echo "variant $v"; cat gpurun_out/wg_${TAG}_$v.log; done
