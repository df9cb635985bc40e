#!/bin/bash
# DiT weight-gradient grouping + side-stream balance: DiT / sampling tests, then same-box step A/Bs and the sampler lines
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_dit_gpu.py tests/test_plan_gpu.py tests/test_dp_gpu.py tests/test_sampling_gpu.py tests/test_rccl_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_r3c.log 2>&1
rc=$?; tail -3 gpurun_out/t_r3c.log; [ $rc -eq 0 ] || exit 1
ms() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['ms_per_step'],3))" $1; }
for r in 1 2; do
  for E in "SDMI_WG_BALANCE=0" "SDMI_WG_BALANCE=1"; do
    env $E timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 30 > gpurun_out/c.log 2>&1 || { tail -5 gpurun_out/c.log; exit 1; }
    echo "cond $E $(ms gpurun_out/c.log)"
  done
  for E in "SDMI_DIT_WG_GROUP=1" "SDMI_DIT_WG_GROUP=3" "SDMI_DIT_WG_GROUP=6"; do
    env $E timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 30 --workload dit > gpurun_out/d.log 2>&1 || { tail -5 gpurun_out/d.log; exit 1; }
    echo "dit $E $(ms gpurun_out/d.log)"
  done
done
for smp in ddpm ddim; do
  timeout -k 10 300 python -u bench.py --workload sample --sampler $smp --steps 50 --warmup 3 > gpurun_out/s_$smp.log 2>&1 || { tail -5 gpurun_out/s_$smp.log; exit 1; }
  tail -1 gpurun_out/s_$smp.log | cut -c1-200; python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['ms_per_step'], d['roofline'])" gpurun_out/s_$smp.log
done
