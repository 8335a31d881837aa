#!/bin/bash
# C++ cast node on the HF-swap path: tests, phases, Python-cast vs C++-cast A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_llama.py tests/test_gpu_block_graphs.py -x -q --timeout 200 --timeout-method thread > gpurun_out/llama_tests2.txt 2>&1 &&
timeout -k 10 240 python -u benchmarks/notebook_step.py --modes hfnativedefault --steps 30 --warm 6 --phases > gpurun_out/hfnative_cast.txt 2>&1 &&
for r in 1 2 3; do
  NBD_NATIVE_CAST=0 timeout -k 10 240 python -u benchmarks/notebook_step.py --modes hfnativedefault --steps 40 --warm 6 | sed 's/^hfnativedefault/pycast /' || exit $?
  timeout -k 10 240 python -u benchmarks/notebook_step.py --modes hfnativedefault --steps 40 --warm 6 | sed 's/^hfnativedefault/cppcast/' || exit $?
done >> gpurun_out/hfnative_cast.txt 2>&1
