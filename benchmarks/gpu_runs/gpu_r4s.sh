#!/bin/bash
# the one-line HF swap (nbd.models.native) with and without per-block forward graphs
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 python -u benchmarks/notebook_step.py --modes hfnative,hfnativebg --steps 30 --warm 6 --phases > gpurun_out/hfnative_phases.txt 2>&1 &&
for r in 1 2 3; do
  timeout -k 10 240 python -u benchmarks/notebook_step.py --modes hfnative,hfnativebg --steps 40 --warm 6 || exit $?
done > gpurun_out/hfnative_ab.txt 2>&1
