#!/bin/bash
# where the runtime copies / fills / torch elementwise kernels sit in the graphed SmolLM2 step
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_nb_seq -o p -- python3 $R/benchmarks/notebook_step.py --modes nbdgraph --steps 8 --warm 4 > $R/gpurun_out/prof_nb_seq.log 2>&1 &&
cd $R && python3 benchmarks/trace_seq.py gpurun_out/prof_nb_seq --pattern 'copyBuffer|fillBuffer|at::native|Cijk' > gpurun_out/nb_seq_r4.txt 2>&1
rm -rf $R/gpurun_out/prof_nb_seq
