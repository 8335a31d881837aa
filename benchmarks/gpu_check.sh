#!/bin/bash
# One GPU call: the GPU test suite, smoke(), then optional extra steps, then bench.py.
#   bash benchmarks/gpu_check.sh [tag] ["extra command"]
set -e
tag=${1:-head}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests_$tag.txt 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$tag.txt 2>&1
if [ -n "$2" ]; then bash -c "$2"; fi
timeout -k 10 300 python bench.py > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err
