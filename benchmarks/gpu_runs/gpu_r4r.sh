#!/bin/bash
# three back-to-back 1-GPU bench.py runs (stability of the eager / graphed arms)
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 420 python -u bench.py > gpurun_out/bench_r4ac$i.json 2> gpurun_out/bench_r4ac$i.log || exit $?
done
