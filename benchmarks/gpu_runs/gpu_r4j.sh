#!/bin/bash
# eager (FlatAdamW overlap) vs eager + per-block forward graphs vs whole-step graph, 5 interleaved rounds
set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3 4 5; do
  NBD_ADAMW_OVERLAP=1 timeout -k 10 240 python -u benchmarks/notebook_step.py --modes nbd,nbdbg,nbdgraph --steps 60 --warm 8 || exit $?
done > gpurun_out/bg_ab5.txt 2>&1
