#!/bin/bash
# kernel trace of the eager step with stack graphs vs the whole-step graph: GPU busy / idle per step
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for m in nbdbg nbdgraph; do
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof2_$m -o run -- python3 benchmarks/notebook_step.py --modes $m --steps 30 --warm 10 > gpurun_out/prof2_$m.log 2>&1 || exit $?
  python3 benchmarks/trace_gaps.py gpurun_out/prof2_$m --steps 10 > gpurun_out/gaps2_$m.txt 2>&1 || exit $?
done
rm -rf gpurun_out/prof2_*/
