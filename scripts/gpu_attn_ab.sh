#!/bin/bash
# Attention kernels: parity tests, isolated timing of the working tree vs the library in abprev/ (same box), then the
# SQ counters (bank conflicts) of the working tree at one shape (SHAPE, default 2 = 32^2 self-attention d = 24).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_unet_gpu.py tests/test_dit_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_attn.log 2>&1
rc=$?; tail -3 gpurun_out/t_attn.log; [ $rc -eq 0 ] || exit 1
for r in 1 2; do
  SDMI_LIB_PATH=$GRAFT_REPO_ROOT/abprev/stablediffusion-pytorch_amd/sdmi/libsdmi.so timeout -k 10 120 python -u scripts/attn_bench.py > gpurun_out/attn_old$r.txt 2>&1 || exit 1
  timeout -k 10 120 python -u scripts/attn_bench.py > gpurun_out/attn_new$r.txt 2>&1 || exit 1
done
paste gpurun_out/attn_old2.txt gpurun_out/attn_new2.txt
SHAPE=${SHAPE:-2} bash scripts/gpu_attn_pmc.sh
