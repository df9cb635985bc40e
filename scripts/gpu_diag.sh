#!/bin/bash
# Attribution of the overlapped step: the headline bench with the weight-gradient GEMMs and / or the optimizer left
# out (SDMI_DIAG_SKIP; diagnostic numbers only, the step then trains wrongly)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for sk in "" wg opt wg,opt "" ; do
  SDMI_DIAG_SKIP=$sk timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/b_diag.log 2>&1 || { tail -20 gpurun_out/b_diag.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/b_diag.log').read().strip().splitlines()[-1]);print('skip=$sk', round(d['ms_per_step'],3))"
done
