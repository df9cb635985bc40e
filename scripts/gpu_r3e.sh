#!/bin/bash
# Session-5 GPU pass: the sampling-step probe (plan replay vs one hipGraph, B = 1 / 8, context branch inline or on
# its own stream), the -m gpu suite on the current tree, the headline bench.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for B in 1 8; do
  for CS in 0 1; do
    SDMI_CTX_STREAM=$CS timeout -k 10 180 python -u scripts/sample_graph_probe.py $B >> gpurun_out/sg_r3e.log 2>&1 || { tail -20 gpurun_out/sg_r3e.log; exit 1; }
  done
done
grep "B=" gpurun_out/sg_r3e.log
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -rf > gpurun_out/t_r3e.log 2>&1
rc=$?; tail -8 gpurun_out/t_r3e.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "pytest rc=$rc"; exit $rc; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/b_r3e.log 2>&1 || { tail -20 gpurun_out/b_r3e.log; exit 1; }
tail -1 gpurun_out/b_r3e.log | cut -c1-300
