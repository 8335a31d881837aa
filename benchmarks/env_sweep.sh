#!/bin/bash
# Sweep of environment settings on the GPT-2 small DDP step (eager + one HIP graph), interleaved
# processes on one box:  ROUNDS=2 bash benchmarks/env_sweep.sh "NBD_X=a" "NBD_X=b" "NBD_X=c" ...
set -e
rounds=${ROUNDS:-2}
for i in $(seq 1 "$rounds"); do
  for e in "$@"; do
    echo "== $e round $i"
    env $e timeout -k 10 300 python benchmarks/ddp_compare.py --impls flat,flatgraph --rounds 2 --steps 10
  done
done
