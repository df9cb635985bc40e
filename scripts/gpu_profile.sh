#!/bin/bash
# Closing profile of one workload on the current tree: isolated per-op plan profile, rocprofv3 kernel trace + stats,
# PMC HBM traffic (separate FETCH_SIZE / WRITE_SIZE passes) and the roofline evidence of the kernel the bench line
# itself names (roofline.kernel_id / launch_set), all tagged with the tree's source digest. Outputs:
# (WL = cond-unet | dit | uncond-unet | vqvae | vqvae-train)
# gpurun_out/<TAG>_<wl>_pmc_traffic.json and gpurun_out/<TAG>_<wl>_roofline_evidence.json -- copied to profiles/ as
# rNN_<wl>_*.json, where bench.py finds them (and reports whether they were measured on the running tree).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-prof}
WL=${WL:-cond-unet}
W=${WL//-/_}
mkdir -p gpurun_out
DIG=$(python3 stablediffusion-pytorch_amd/sdmi/_build.py --digest)
timeout -k 10 300 python -u bench.py --no-cpu-baseline --workload $WL > gpurun_out/bench_${TAG}_$W.log 2>&1 || { tail -20 gpurun_out/bench_${TAG}_$W.log; exit 1; }
tail -1 gpurun_out/bench_${TAG}_$W.log > gpurun_out/${TAG}_${W}_bench.json
ROOF_KERNEL=$(python3 -c "import json,sys; print(json.load(open(sys.argv[1]))['roofline']['kernel_id'])" gpurun_out/${TAG}_${W}_bench.json)
LAUNCHES=$(python3 -c "import json,sys; print(json.load(open(sys.argv[1]))['roofline']['launch_set'])" gpurun_out/${TAG}_${W}_bench.json)
echo "digest $DIG roofline kernel: $ROOF_KERNEL ($LAUNCHES launches)"
if [[ $WL != vqvae* ]]; then  # (the isolated plan profile covers the recorded training steps of the denoisers)
  PLAN_PROFILE_JSON=gpurun_out/pp_${TAG}_$W.json timeout -k 10 400 python -u scripts/plan_profile.py --workload $WL --top 120 > gpurun_out/pp_${TAG}_$W.txt 2>&1 || { tail -20 gpurun_out/pp_${TAG}_$W.txt; exit 1; }
  head -3 gpurun_out/pp_${TAG}_$W.txt
fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG}_$W -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --workload $WL > gpurun_out/prof_${TAG}_$W.log 2>&1 || { tail -20 gpurun_out/prof_${TAG}_$W.log; exit 1; }
MARK=add_noise_kernel; [[ $WL == vqvae* ]] && MARK=prep_input_kernel  # the first launch of a VQVAE step
python scripts/trace_summary.py gpurun_out/prof_${TAG}_$W/run_kernel_trace.csv --top 80 --marker $MARK > gpurun_out/ts_${TAG}_$W.txt
head -8 gpurun_out/ts_${TAG}_$W.txt
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/pmc_${TAG}_${W}_$C -o run -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --issue eager --workload $WL > gpurun_out/pmc_${TAG}_${W}_$C.log 2>&1 || { tail -5 gpurun_out/pmc_${TAG}_${W}_$C.log; exit 1; }
done
python3 scripts/pmc_summary.py gpurun_out/pmc_${TAG}_${W}_FETCH_SIZE gpurun_out/pmc_${TAG}_${W}_WRITE_SIZE --json gpurun_out/${TAG}_${W}_pmc_traffic.json --meta $WL $DIG > gpurun_out/pmc_${TAG}_$W.txt
head -12 gpurun_out/pmc_${TAG}_$W.txt
python3 scripts/roofline_evidence.py gpurun_out/prof_${TAG}_$W gpurun_out/pmc_${TAG}_${W}_FETCH_SIZE gpurun_out/pmc_${TAG}_${W}_WRITE_SIZE "$ROOF_KERNEL" --launches $LAUNCHES --meta $WL $DIG --json gpurun_out/${TAG}_${W}_roofline_evidence.json
