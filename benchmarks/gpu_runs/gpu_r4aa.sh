#!/bin/bash
# stack graphs: eager / block graphs with stacks / without stacks / whole-step graph; HF swap
set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3 4; do
  timeout -k 10 240 python -u benchmarks/notebook_step.py --modes nbd,nbdbg,nbdgraph --steps 60 --warm 10 || exit $?
  NBD_BLOCK_STACKS=0 timeout -k 10 240 python -u benchmarks/notebook_step.py --modes nbdbg --steps 60 --warm 10 | sed 's/^nbdbg /nbdbg-nostack /' || exit $?
  timeout -k 10 240 python -u benchmarks/notebook_step.py --modes hfnativedefault --steps 60 --warm 10 || exit $?
done > gpurun_out/stack_ab_box2.txt 2>&1 &&
timeout -k 10 240 python -u benchmarks/notebook_step.py --modes nbdbg --steps 30 --warm 10 --phases > gpurun_out/stack_phases_box2.txt 2>&1
