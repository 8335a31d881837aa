#!/bin/bash
# Sweep of environment settings on the SmolLM2 notebook step (eager + one HIP graph), interleaved
# processes on one box:  ROUNDS=2 bash benchmarks/nb_env_sweep.sh "NBD_X=a" "NBD_X=b" ...
set -e
rounds=${ROUNDS:-2}
for i in $(seq 1 "$rounds"); do
  for e in "$@"; do
    echo "== $e round $i"
    env $e timeout -k 10 200 python benchmarks/notebook_step.py --modes nbd,nbdgraph --steps 30
  done
done
