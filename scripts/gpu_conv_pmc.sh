#!/bin/bash
# SQ counters of the 32^2 conv forward vs weight-gradient mainloops (scripts/conv_pmc_probe.py), one pass per counter set
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for C in ${CASES:-fwd wg1v2 wg6v2 wg3v11 wg1v1}; do
  timeout -k 10 60 python3 scripts/conv_pmc_probe.py $C 2>&1 | grep -v amdgpu
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS --output-format csv -d gpurun_out/cpmc1_$C -o run -- python3 scripts/conv_pmc_probe.py $C > gpurun_out/cpmc1_$C.log 2>&1 || { tail -5 gpurun_out/cpmc1_$C.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU_TRANS_F32 SQ_WAVES --output-format csv -d gpurun_out/cpmc2_$C -o run -- python3 scripts/conv_pmc_probe.py $C > gpurun_out/cpmc2_$C.log 2>&1 || { tail -5 gpurun_out/cpmc2_$C.log; exit 1; }
  python3 - $C <<'PY'
import csv, glob, collections, sys
c = sys.argv[1]
for d in (f"gpurun_out/cpmc1_{c}", f"gpurun_out/cpmc2_{c}"):
    f = glob.glob(d + "/**/*counter_collection.csv", recursive=True)
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f[0])):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:64]
        if "gemm" not in k and "splitk" not in k: continue
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in acc.items():
        print(c, k, {n: "%.4g" % (sum(v) / len(v)) for n, v in cs.items()})
PY
done
