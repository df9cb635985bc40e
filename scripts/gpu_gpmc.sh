#!/bin/bash
# PMC passes over scripts/gemm_pmc_probe.py (one counter group per pass)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-gp}
timeout -s KILL 60 rocprofv3 -L > gpurun_out/pmc_list.txt 2>&1 || true
i=0
for C in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE" "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA TA_BUSY_max TA_TA_BUSY_sum"; do
  timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/gp_${TAG}_$i -o run -- python3 scripts/gemm_pmc_probe.py > gpurun_out/gp_${TAG}_$i.log 2>&1 || { echo "pass $i failed"; tail -3 gpurun_out/gp_${TAG}_$i.log; }
  i=$((i+1))
done
ls gpurun_out/gp_${TAG}_*/
