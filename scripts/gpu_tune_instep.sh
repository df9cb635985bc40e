#!/bin/bash
# In-step GEMM table re-tune (scripts/tune_in_step.py) of one workload, then a same-box bench A/B of the new table
# against the package's on the workloads that share its shapes.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
WL=${WL:-cond-unet}
timeout -k 10 700 python -u scripts/tune_in_step.py --workload $WL --keys ${KEYS:-14} --out gpurun_out/tuned_instep.json > gpurun_out/tune_instep_$WL.log 2>&1 || { tail -30 gpurun_out/tune_instep_$WL.log; exit 1; }
grep -c KEEP gpurun_out/tune_instep_$WL.log; tail -3 gpurun_out/tune_instep_$WL.log
ARMS=".;SDMI_TUNED_GEMM=gpurun_out/tuned_instep.json" WLS="${ABWLS:-cond-unet uncond-unet dit}" bash scripts/gpu_env_ab.sh
