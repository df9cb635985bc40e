#!/bin/bash
# Attention forward with the MFMA-side scale / max offset and lazy rebase (SDMI_ATTN_LAZY=1) and the pre-scaled backward (bit 2): kernel and model parity
# tests under it, isolated kernel times against the default kernel, then a same-box A/B of the headline step
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
SDMI_ATTN_LAZY=3 timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_unet_gpu.py tests/test_dit_gpu.py tests/test_cabi_gpu.py -q --timeout 200 --timeout-method thread -rf > gpurun_out/t_lazy.log 2>&1
rc=$?; tail -6 gpurun_out/t_lazy.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
for A in 1 3; do
  ATTN_AMP=$A timeout -k 10 120 python -u scripts/attn_bench.py > gpurun_out/ab_base.txt 2>&1 || { tail gpurun_out/ab_base.txt; exit 1; }
  SDMI_ATTN_LAZY=3 ATTN_AMP=$A timeout -k 10 120 python -u scripts/attn_bench.py > gpurun_out/ab_lazy.txt 2>&1 || { tail gpurun_out/ab_lazy.txt; exit 1; }
  echo "amp $A base"; grep "B=" gpurun_out/ab_base.txt | cut -c1-100
  echo "amp $A lazy=3"; grep "B=" gpurun_out/ab_lazy.txt | cut -c1-100
done
ENVS="SDMI_ATTN_LAZY=1;SDMI_ATTN_LAZY=3" ROUNDS=2 bash scripts/gpu_envab.sh
