#!/bin/bash
# Same-box A/B of the step's issue modes: native plan replay on 4 streams (default) vs single-stream hipGraph
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
ms() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['ms_per_step'],3))" $1; }
for r in 1 2; do
  for I in plan graph; do
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 30 --issue $I > gpurun_out/issue_$I$r.log 2>&1 || { tail -5 gpurun_out/issue_$I$r.log; exit 1; }
    echo "issue=$I r$r $(ms gpurun_out/issue_$I$r.log)"
  done
done
