#!/bin/bash
# A/B of an environment setting on the GPT-2 small DDP step (eager + one HIP graph), interleaved
# processes on one box:
#   bash benchmarks/env_ab.sh "NBD_X=a" "NBD_X=b" [rounds]
set -e
A=$1
B=$2
rounds=${3:-2}
for i in $(seq 1 "$rounds"); do
  echo "== A ($A) round $i"
  env $A timeout -k 10 300 python benchmarks/ddp_compare.py --impls flat,flatgraph --rounds 2 --steps 10
  echo "== B ($B) round $i"
  env $B timeout -k 10 300 python benchmarks/ddp_compare.py --impls flat,flatgraph --rounds 2 --steps 10
done
