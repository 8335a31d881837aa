#!/bin/bash
# where the runtime copies / fills sit in the graphed GPT-2 step (kernel before / after each)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_gpt2_seq -o p -- python3 $R/benchmarks/ddp_compare.py --impls flatgraph --rounds 1 --steps 6 --warm 3 > $R/gpurun_out/prof_gpt2_seq.log 2>&1 &&
cd $R && python3 benchmarks/trace_seq.py gpurun_out/prof_gpt2_seq --pattern 'copyBuffer|fillBuffer|bfloat16_copy|FillFunctor|elementwise' > gpurun_out/gpt2_seq_r4.txt 2>&1
rm -rf $R/gpurun_out/prof_gpt2_seq
