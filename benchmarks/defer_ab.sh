#!/bin/bash
# Deferred weight-gradient reduces (NBD_GRAD_DEFER) A/B: the GPU test suite, then the SmolLM2
# notebook step and the GPT-2 step (eager + one HIP graph), interleaved processes.
#   bash benchmarks/defer_ab.sh [tag] [rounds]
set -e
tag=${1:-now}
rounds=${2:-2}
mkdir -p gpurun_out
o=gpurun_out/defer_ab_$tag.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/defer_tests_$tag.txt 2>&1
: > $o
for i in $(seq 1 "$rounds"); do
  for e in NBD_GRAD_DEFER=0 NBD_GRAD_DEFER=1; do
    echo "== $e round $i" >> $o
    env $e timeout -k 10 200 python benchmarks/notebook_step.py --modes nbd,nbdgraph --steps 30 >> $o 2>&1
    env $e timeout -k 10 300 python benchmarks/ddp_compare.py --impls flat,flatgraph --rounds 2 --steps 10 >> $o 2>&1
  done
done
