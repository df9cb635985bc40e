#!/bin/bash
# Which hardware queue each stream lands on (rocprofv3 kernel trace Queue_Id), and the step time, for the plain and the
# forced-reducer step under stream-priority arms (ARMS as in gpu_env_ab.sh)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
ARMS="${ARMS:-.;SDMI_MAIN_PRIORITY=high;SDMI_SIDE_PRIORITY=-1}"
BARGS=--force-reducer ARMS="$ARMS" bash scripts/gpu_env_ab.sh || exit 1
for f in gpurun_out/envab_cond-unet_*.log; do cp $f ${f%.log}.forced.log; done
ARMS="$ARMS" bash scripts/gpu_env_ab.sh || exit 1
IFS=';' read -ra A <<< "$ARMS"
i=0
for E in "${A[@]}"; do
  i=$((i+1)); if [ "$E" = "." ]; then EE=""; else EE="$E"; fi
  for BA in --force-reducer ""; do
    d=gpurun_out/q_$i${BA:+f}
    env $EE timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline $BA > $d.log 2>&1 || { tail -20 $d.log; exit 1; }
    python3 - $d "$E $BA" <<'PY'
import csv, collections, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
c = collections.Counter((int(r["Stream_Id"]), int(r["Queue_Id"])) for r in rows)
print(sys.argv[2], "stream:queue(dispatches)", " ".join(f"{s}:{q}({n})" for (s, q), n in sorted(c.items())))
PY
  done
done
