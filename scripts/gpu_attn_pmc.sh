#!/bin/bash
# SQ counters of the attention kernels at the 32^2 self-attention shape
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS --output-format csv -d gpurun_out/apmc1 -o run -- python3 scripts/attn_bench.py ${SHAPE:-0} > gpurun_out/apmc1.log 2>&1 || { tail -5 gpurun_out/apmc1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU_TRANS_F32 SQ_WAVES --output-format csv -d gpurun_out/apmc2 -o run -- python3 scripts/attn_bench.py ${SHAPE:-0} > gpurun_out/apmc2.log 2>&1 || { tail -5 gpurun_out/apmc2.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
for d in ("gpurun_out/apmc1", "gpurun_out/apmc2"):
    f = glob.glob(d + "/**/*counter_collection.csv", recursive=True)
    if not f:
        print("no counter file in", d); continue
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f[0])):
        k = r["Kernel_Name"][:40]
        if "attn" not in k: continue
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in acc.items():
        print(k, {c: "%.3g" % (sum(v) / len(v)) for c, v in cs.items()})
PY
