cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
SDMI_GN_DEFER=1 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_u.log 2>&1
rc=$?; tail -2 gpurun_out/t_u.log; [ $rc -eq 0 ] || exit 1
ARMS=". .:SDMI_GN_DEFER=1" bash scripts/gpu_bisect.sh || exit 1
cp stablediffusion-pytorch_amd/sdmi/tuned_gemm.json gpurun_out/tuned_s.json
for SB in 1 8; do
  SDMI_TUNE_VARIANTS=9,10 timeout -k 10 600 python -u scripts/tune_gemm.py --workload sample --sample-batch $SB --against-table --out gpurun_out/tuned_s.json > gpurun_out/tune_s$SB.log 2>&1 || { tail -5 gpurun_out/tune_s$SB.log; exit 1; }
  tail -2 gpurun_out/tune_s$SB.log
done
ms() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['ms_per_step'],3))" $1; }
for r in 1 2; do
  for SB in 1 8; do
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --workload sample --sample-batch $SB --steps 40 > gpurun_out/s_base_$SB$r.log 2>&1 || exit 1
    SDMI_TUNED_GEMM=gpurun_out/tuned_s.json timeout -k 10 300 python -u bench.py --no-cpu-baseline --workload sample --sample-batch $SB --steps 40 > gpurun_out/s_new_$SB$r.log 2>&1 || exit 1
    echo "sample B=$SB r$r base $(ms gpurun_out/s_base_$SB$r.log) new $(ms gpurun_out/s_new_$SB$r.log)"
  done
done
