#!/bin/bash
# HF swap with kept cast buffers: tests; the notebook's lines (+ native()) with and without block graphs
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_block_graphs.py tests/test_gpu_llama.py -x -q --timeout 200 --timeout-method thread > gpurun_out/bg_tests4.txt 2>&1 &&
timeout -k 10 240 python -u benchmarks/notebook_step.py --modes hfnativedefault,hfnativebg --steps 30 --warm 6 --phases > gpurun_out/hfnative_bg2.txt 2>&1 &&
for r in 1 2 3 4; do
  timeout -k 10 240 python -u benchmarks/notebook_step.py --modes hfnativedefault,hfnativebg --steps 40 --warm 6 || exit $?
done >> gpurun_out/hfnative_bg2.txt 2>&1
