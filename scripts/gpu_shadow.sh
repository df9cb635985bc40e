#!/bin/bash
# bf16 parameter image (SDMI_SHADOW): trainer / plan / DP parity tests, then a same-box A/B of the headline step and
# the DiT step (SDMI_SHADOW=1 vs 0, alternating), then the attention kernels at the model's shapes.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_plan_gpu.py tests/test_unet_gpu.py tests/test_dit_gpu.py tests/test_dp_gpu.py tests/test_gradscaler_gpu.py tests/test_bench_step_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_shadow.log 2>&1
rc=$?; tail -3 gpurun_out/t_shadow.log; [ $rc -eq 0 ] || exit 1
ms() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['ms_per_step'],3))" $1; }
for r in 1 2; do
  for sh in 0 1; do
    SDMI_SHADOW=$sh timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 30 > gpurun_out/sh$sh.log 2>&1 || { tail -5 gpurun_out/sh$sh.log; exit 1; }
    echo "cond shadow=$sh $(ms gpurun_out/sh$sh.log)"
  done
done
for r in 1 2; do
  for sh in 0 1; do
    SDMI_SHADOW=$sh timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 30 --workload dit > gpurun_out/shd$sh.log 2>&1 || { tail -5 gpurun_out/shd$sh.log; exit 1; }
    echo "dit shadow=$sh $(ms gpurun_out/shd$sh.log)"
  done
done
timeout -k 10 300 python -u scripts/attn_bench.py > gpurun_out/attn_shapes.txt 2>&1 || { tail -5 gpurun_out/attn_shapes.txt; exit 1; }
cat gpurun_out/attn_shapes.txt
