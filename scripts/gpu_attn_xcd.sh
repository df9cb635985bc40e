#!/bin/bash
# Attention A/B of two libraries (abprev/libsdmi.so vs the tree's): isolated timing at every shape, then PMC HBM
# traffic (FETCH_SIZE / WRITE_SIZE passes) per attention kernel at the 32^2 d = 24 self-attention (shape 2).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
T=${TAG:-attn}
OLD=$GRAFT_REPO_ROOT/abprev/libsdmi.so
for r in 1 2; do
  SDMI_LIB_PATH=$OLD timeout -k 10 120 python -u scripts/attn_bench.py > gpurun_out/${T}_old$r.txt 2>&1 || exit 1
  timeout -k 10 120 python -u scripts/attn_bench.py > gpurun_out/${T}_new$r.txt 2>&1 || exit 1
done
for which in old new; do
  for C in FETCH_SIZE WRITE_SIZE; do
    if [ $which = old ]; then export SDMI_LIB_PATH=$OLD; else unset SDMI_LIB_PATH; fi
    timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/${T}_pmc_${which}_$C -o run -- python3 scripts/attn_bench.py ${SHAPE:-2} > gpurun_out/${T}_pmc_${which}_$C.log 2>&1 || { tail -5 gpurun_out/${T}_pmc_${which}_$C.log; exit 1; }
  done
  unset SDMI_LIB_PATH
  python3 scripts/pmc_summary.py gpurun_out/${T}_pmc_${which}_FETCH_SIZE gpurun_out/${T}_pmc_${which}_WRITE_SIZE > gpurun_out/${T}_pmc_$which.txt
done
for r in 1 2; do echo "== old $r"; cat gpurun_out/${T}_old$r.txt | grep B=; echo "== new $r"; cat gpurun_out/${T}_new$r.txt | grep B=; done
for which in old new; do echo "== PMC $which"; grep -i attn gpurun_out/${T}_pmc_$which.txt; done
