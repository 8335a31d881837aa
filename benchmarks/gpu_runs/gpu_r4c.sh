#!/bin/bash
# round-4 batch: LM-head products on the 256 kernel vs hipBLASLt; K3 no_sync A/B; GPT-2 graphed vs
# eager over back-to-back bench runs (the capture-safe warm-up must not make the graph slower)
set -e
mkdir -p gpurun_out
timeout -k 10 180 python benchmarks/lmhead_hip_ab.py > gpurun_out/lmhead_hip_ab_r4.txt 2>&1
bash benchmarks/ab_lib.sh gpurun_ab/libnbd_ops_base.so "python benchmarks/ops_bench.py --only prereduce" 2 > gpurun_out/k3_ab_r4.txt 2>&1
for i in 1 2 3 4 5 6; do
  timeout -k 10 200 python bench.py --no-notebook --no-bcast --no-sweep --steps 20 --warmup 5 > gpurun_out/bench6_$i.json 2> gpurun_out/bench6_$i.err
done
