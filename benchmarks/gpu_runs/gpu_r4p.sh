#!/bin/bash
# full GPU suite + smoke + the 1-GPU bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/gputests_r4p.txt 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('__SMOKE_OK__')" > gpurun_out/smoke_r4p.txt 2>&1 &&
timeout -k 10 600 python -u bench.py > gpurun_out/bench_r4p.json 2> gpurun_out/bench_r4p.log
