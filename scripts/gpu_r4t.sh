cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
SDMI_EAGER_WG=1 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_t.log 2>&1
rc=$?; tail -2 gpurun_out/t_t.log; [ $rc -eq 0 ] || exit 1
ARMS=".:SDMI_TUNED_GEMM=$GRAFT_REPO_ROOT/abtmp/tuned_prev.json . .:SDMI_EAGER_WG=1" bash scripts/gpu_bisect.sh || exit 1
ms() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['ms_per_step'],3))" $1; }
for r in 1 2; do
  SDMI_TUNED_GEMM=$GRAFT_REPO_ROOT/abtmp/tuned_prev.json timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 30 --workload dit > gpurun_out/dit_prev$r.log 2>&1 || exit 1
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 30 --workload dit > gpurun_out/dit_new$r.log 2>&1 || exit 1
  echo "dit r$r prev $(ms gpurun_out/dit_prev$r.log) new $(ms gpurun_out/dit_new$r.log)"
done
