#!/bin/bash
# A/B of environment knobs on the eager bench: each line of $VARIANTS is an env assignment list.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
while read -r v; do
  [ -z "$v" ] && continue
  r=$(env $v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],3))")
  echo "$v -> $r ms/step"
done <<< "$VARIANTS"
