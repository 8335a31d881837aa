#!/bin/bash
# kernel traces of the eager / block-graphed / whole-graph notebook steps: GPU idle per step
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for m in nbd nbdbg nbdbg2 nbdgraph; do
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_$m -o run -- python3 benchmarks/notebook_step.py --modes $m --steps 20 --warm 6 > gpurun_out/prof_$m.log 2>&1 || exit $?
  python3 benchmarks/trace_gaps.py gpurun_out/prof_$m --steps 10 > gpurun_out/gaps_$m.txt 2>&1 || exit $?
done
rm -rf gpurun_out/prof_*/
