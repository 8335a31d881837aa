#!/bin/bash
# HF swap: torch AdamW foreach (the notebook's line) vs fused=True; block-graph tests after the leaf rule
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_block_graphs.py -x -q --timeout 200 --timeout-method thread > gpurun_out/bg_tests3.txt 2>&1 &&
timeout -k 10 240 python -u benchmarks/notebook_step.py --modes hfnative,hfnativefused --steps 30 --warm 6 --phases > gpurun_out/hfnative_fused.txt 2>&1 &&
for r in 1 2; do
  timeout -k 10 240 python -u benchmarks/notebook_step.py --modes hfnative,hfnativefused,hfnativebg --steps 40 --warm 6 || exit $?
done >> gpurun_out/hfnative_fused.txt 2>&1
