#!/bin/bash
# block graphs (mode 2 with recorded deferred reductions): tests, phase/host timing, 4-mode A/B; K3 acc shapes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_block_graphs.py tests/test_gpu_llama_block.py -x -v --timeout 200 --timeout-method thread > gpurun_out/bg_tests.txt 2>&1 &&
NBD_HOST_TIMING=1 timeout -k 10 240 python -u benchmarks/notebook_step.py --modes nbd,nbdbg,nbdbg2 --steps 30 --warm 6 --phases > gpurun_out/host_timing.txt 2>&1 &&
for r in 1 2 3 4 5; do
  timeout -k 10 240 python -u benchmarks/notebook_step.py --modes nbd,nbdbg,nbdbg2,nbdgraph --steps 60 --warm 8 || exit $?
done > gpurun_out/bg_ab5n.txt 2>&1 &&
bash benchmarks/gpu_r4m.sh
