#!/bin/bash
# per-block HIP graphs: GPU tests + eager / block-graphed / whole-step-graphed notebook step A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_block_graphs.py tests/test_gpu_llama_block.py -x -v --timeout 200 --timeout-method thread > gpurun_out/bg_tests.txt 2>&1 &&
for r in 1 2 3; do
  timeout -k 10 240 python -u benchmarks/notebook_step.py --modes nbd,nbdbg,nbdbg2,nbdgraph --steps 40 --warm 6 || exit $?
done > gpurun_out/bg_ab.txt 2>&1
