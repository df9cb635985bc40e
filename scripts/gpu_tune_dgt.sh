#!/bin/bash
# Tune the GEMM table with transposed linear dgrad weights (SDMI_DGRAD_T=1: dgrads become B_NK GEMMs that can take
# the 64-row deep-ring tiles), then A/B the step against the default (DGRAD_T=0, committed table).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
cp stablediffusion-pytorch_amd/sdmi/tuned_gemm.json gpurun_out/tuned_dgt.json
SDMI_DGRAD_T=1 timeout -k 10 900 python -u scripts/tune_gemm.py --out gpurun_out/tuned_dgt.json > gpurun_out/tune_dgt.log 2>&1 || { tail -20 gpurun_out/tune_dgt.log; exit 1; }
tail -2 gpurun_out/tune_dgt.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/b_dgt_A$i.log 2>&1 || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/b_dgt_A$i.log').read().strip().splitlines()[-1]);print('A dgrad_t=0', d['ms_per_step'])"
  SDMI_DGRAD_T=1 SDMI_TUNED_GEMM=gpurun_out/tuned_dgt.json timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/b_dgt_B$i.log 2>&1 || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/b_dgt_B$i.log').read().strip().splitlines()[-1]);print('B dgrad_t=1', d['ms_per_step'])"
done
