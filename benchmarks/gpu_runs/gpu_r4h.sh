#!/bin/bash
# round-4 profiles (GPT-2 graphed step, notebook graphed step) and the eager notebook step:
# C++ bucket hooks on / off, eager vs graphed over several processes
set -e
mkdir -p gpurun_out
bash benchmarks/prof_gpt2_graph.sh
bash benchmarks/prof_notebook.sh
for i in 1 2 3; do
  echo "== cpp hooks on $i"; NBD_ADAMW_OVERLAP=1 timeout -k 10 200 python benchmarks/notebook_step.py --modes nbd,nbdgraph --steps 40 2>&1 | grep "nbd"
  echo "== cpp hooks off $i"; NBD_DDP_CPP_HOOKS=0 NBD_ADAMW_OVERLAP=1 timeout -k 10 200 python benchmarks/notebook_step.py --modes nbd --steps 40 2>&1 | grep "nbd"
done > gpurun_out/nb_eager_hooks_r4.txt 2>&1
