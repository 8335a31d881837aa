#!/bin/bash
set -e
mkdir -p gpurun_out
for i in 1 2; do echo "== warm=1 process $i"; timeout -k 10 200 python benchmarks/graph_first_diag.py; done > gpurun_out/graph_first_diag.txt 2>&1
for i in 1 2; do echo "== warm=0 process $i"; NBD_GEMM_WARM=0 timeout -k 10 200 python benchmarks/graph_first_diag.py; done >> gpurun_out/graph_first_diag.txt 2>&1
