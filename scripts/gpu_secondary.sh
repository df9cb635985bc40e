#!/bin/bash
# Secondary bench lines of the round (DiT-12L step, captured DDPM / DDIM sampling at B = 1 and 8, uncond UNet, VQVAE
# encode + decode and training (BASELINE config 2), the headline step with the N > 1 reducer forced on at N = 1)
# and the bf16-wire rehearsal kernel traces (1 vs 3 steps): one JSON line each into gpurun_out/<tag>_bench_*.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${TAG:-r04}
run() {  # name, bench args
  local n=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/${T}_bench_$n.log 2>&1 || { tail -5 gpurun_out/${T}_bench_$n.log; return 1; }
  tail -1 gpurun_out/${T}_bench_$n.log > gpurun_out/${T}_bench_$n.json
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],3), 'ms')" gpurun_out/${T}_bench_$n.json $n
}
run dit --workload dit && run sample_1 --workload sample --steps 40 && run sample_8 --workload sample --sample-batch 8 --steps 40 \
  && run sample_ddim --workload sample --sampler ddim --steps 40 && run uncond_unet --workload uncond-unet \
  && run vqvae --workload vqvae && run vqvae_train --workload vqvae-train --steps 10 \
  && run cond_forced_reducer --force-reducer || exit 1
for S in 1 3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/wire_$S -o run -- python3 scripts/wire_rehearsal.py $S bf16 > gpurun_out/wire_$S.log 2>&1 || { tail -5 gpurun_out/wire_$S.log; exit 1; }
done
python3 - <<'PY'
import csv, collections
c = {}
for S in (1, 3):
    k = collections.Counter(r["Kernel_Name"].split("(")[0][:80] for r in csv.DictReader(open(f"gpurun_out/wire_{S}/run_kernel_trace.csv")))
    c[S] = k
extra = {n: c[3][n] - c[1].get(n, 0) for n in c[3] if c[3][n] != c[1].get(n, 0)}
aten = {n: v for n, v in extra.items() if "at::" in n}
print("kernels added by 2 more bf16-wire steps:", sum(extra.values()), "of which aten:", aten)
PY
