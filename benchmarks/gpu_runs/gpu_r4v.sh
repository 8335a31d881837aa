#!/bin/bash
# HF swap: the notebook's optimizer line as written (native() makes it fused) vs explicit foreach / fused
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 240 python -u benchmarks/notebook_step.py --modes hfnative,hfnativedefault,hfnativefused --steps 40 --warm 6 || exit $?
done > gpurun_out/hfnative_default.txt 2>&1
