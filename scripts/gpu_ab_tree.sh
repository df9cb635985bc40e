#!/bin/bash
# A/B of python-only changes on one box: tests, then the headline bench alternating between a copy of the tree whose
# sdmi/*.py are replaced by the files in ab_old/ (populate it with `git show <rev>:<path> > ab_old/<file>`) and the
# current tree.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u -m pytest tests/test_unet_gpu.py tests/test_plan_gpu.py tests/test_dp_gpu.py tests/test_rccl_gpu.py tests/test_module_gpu.py tests/test_leaf_gpu.py tests/test_latent_gen_gpu.py tests/test_sampling_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_cb.log 2>&1; rc=$?; tail -3 gpurun_out/t_cb.log; [ $rc -eq 0 ] || exit 1
mkdir -p /tmp/abold && cp -r bench.py stablediffusion-pytorch_amd tests oracle profiles /tmp/abold/ && cp ab_old/*.py /tmp/abold/stablediffusion-pytorch_amd/sdmi/
for r in 1 2; do
  (cd /tmp/abold && timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 30 > $GRAFT_REPO_ROOT/gpurun_out/cb_old$r.log 2>&1) || { tail -5 gpurun_out/cb_old$r.log; exit 1; }
  echo "old$r $(tail -1 gpurun_out/cb_old$r.log | python3 -c 'import json,sys; print(round(json.loads(sys.stdin.read())["ms_per_step"],3))')"
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 30 > gpurun_out/cb_new$r.log 2>&1 || { tail -5 gpurun_out/cb_new$r.log; exit 1; }
  echo "new$r $(tail -1 gpurun_out/cb_new$r.log | python3 -c 'import json,sys; print(round(json.loads(sys.stdin.read())["ms_per_step"],3))')"
done
