#!/bin/bash
# accumulating-flatten (no_sync pre-reduce) block shapes: correctness + 64 MiB bucket bandwidth
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for v in 0 1 2 3 4; do
    NBD_K3ACC_VARIANT=$v timeout -k 10 120 python -u benchmarks/k3acc_check.py || exit $?
    NBD_K3ACC_VARIANT=$v timeout -k 10 180 python -u benchmarks/ops_bench.py --only prereduce | sed "s/^/v$v /" || exit $?
  done
done > gpurun_out/k3acc_ab.txt 2>&1
