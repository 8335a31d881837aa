#!/bin/bash
# host-time breakdown of the fused Llama block nodes in the eager notebook step
set -o pipefail
mkdir -p gpurun_out
NBD_HOST_TIMING=1 timeout -k 10 240 python -u benchmarks/notebook_step.py --modes nbd,nbdbg,nbdbg2 --steps 30 --warm 6 --phases > gpurun_out/host_timing.txt 2>&1
