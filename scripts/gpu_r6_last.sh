#!/bin/bash
# Last checks of round 6: the parity suite + smoke on the final tree, then the in-step table check of the DiT step.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_last.log 2>&1 || { tail -40 gpurun_out/t_last.log; exit 1; }
tail -1 gpurun_out/t_last.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_last.log 2>&1 || { tail -20 gpurun_out/smoke_last.log; exit 1; }
tail -1 gpurun_out/smoke_last.log
timeout -k 10 600 python -u scripts/tune_in_step.py --workload dit --keys 12 --out gpurun_out/tuned_instep_dit.json > gpurun_out/tune_instep_dit.log 2>&1 || { tail -20 gpurun_out/tune_instep_dit.log; exit 1; }
grep -c KEEP gpurun_out/tune_instep_dit.log; tail -2 gpurun_out/tune_instep_dit.log
