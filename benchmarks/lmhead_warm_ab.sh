#!/bin/bash
# A/B: the LM-head table warmed into the MALL by the last HIP GEMM before the head
# (NBD_LM_HEAD_WARM_MB=0 turns it off), GPT-2 small step eager + graphed, interleaved processes.
set -e
for i in 1 2; do
  echo "== warm off, round $i"
  NBD_LM_HEAD_WARM_MB=0 timeout -k 10 300 python benchmarks/ddp_compare.py --impls flat,flatgraph --rounds 2 --steps 10
  echo "== warm on (96 MB), round $i"
  NBD_LM_HEAD_WARM_MB=96 timeout -k 10 300 python benchmarks/ddp_compare.py --impls flat,flatgraph --rounds 2 --steps 10
done
