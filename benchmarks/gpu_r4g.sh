#!/bin/bash
# BK32 4-stage ring for the grouped backward: correctness, per-shape A/B, GPT-2 step A/B
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py -x -q --timeout 120 --timeout-method thread -k "pair" > gpurun_out/bk32_tests.txt 2>&1
for r in 1 2; do
  echo "== BK64 round $r"; NBD_GEMM_PAIR_BK32=0 timeout -k 10 200 python benchmarks/pair_sched.py --only gpt2 --rounds 2
  echo "== BK32 round $r"; NBD_GEMM_PAIR_BK32=1 timeout -k 10 200 python benchmarks/pair_sched.py --only gpt2 --rounds 2
done > gpurun_out/bk32_pair_ab.txt 2>&1
for r in 1 2; do
  echo "== BK64 round $r"; NBD_GEMM_PAIR_BK32=0 timeout -k 10 200 python benchmarks/graph_first_diag.py flat,flatgraph 2>&1 | grep flat
  echo "== BK32 round $r"; NBD_GEMM_PAIR_BK32=1 timeout -k 10 200 python benchmarks/graph_first_diag.py flat,flatgraph 2>&1 | grep flat
done > gpurun_out/bk32_step_ab.txt 2>&1
