#!/bin/bash
# Eager host cost of the SmolLM2 notebook step: wall vs host-issue time, the torch-profiler and
# cProfile tables, and the step under a few env switches (one GPU call).
#   bash benchmarks/notebook_host.sh [tag]
set -e
tag=${1:-now}
mkdir -p gpurun_out
o=gpurun_out/notebook_host_$tag.txt
: > $o
timeout -k 10 200 python benchmarks/notebook_step.py --modes nbd,nbd --steps 30 >> $o 2>&1
for e in NBD_GEMM_WARM=0; do
  echo "== $e" >> $o
  env $e timeout -k 10 200 python benchmarks/notebook_step.py --modes nbd --steps 30 >> $o 2>&1
done
timeout -k 10 200 python benchmarks/host_profile.py --model smollm2 --steps 5 >> $o 2>&1
timeout -k 10 200 python benchmarks/host_profile.py --model smollm2 --steps 5 --cprofile >> $o 2>&1
bash benchmarks/prof_notebook.sh
