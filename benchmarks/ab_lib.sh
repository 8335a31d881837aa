#!/bin/bash
# A/B two builds of libnbd_ops.so in one GPU call (same box, interleaved runs):
#   bash benchmarks/ab_lib.sh ab/libnbd_ops_base.so "<python benchmark command>" [rounds]
# A = the given library (NBD_OPS_LIB), B = the in-tree nbdistributed_amd/_native/libnbd_ops.so.
set -e
base=$1
cmd=$2
rounds=${3:-2}
for i in $(seq 1 "$rounds"); do
  echo "== A (base: $base) round $i"
  NBD_OPS_LIB=$base timeout -k 10 300 $cmd
  echo "== B (in-tree) round $i"
  timeout -k 10 300 $cmd
done
