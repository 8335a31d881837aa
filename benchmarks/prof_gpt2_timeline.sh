set -e
# rocprofv3 kernel trace of the graphed GPT-2 small flat DDP step -> busy/idle timeline + families
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_tl -o p -- python3 $R/benchmarks/ddp_compare.py --impls ${IMPL:-flatgraph} --rounds 1 --steps 10 --warm 3 > $R/gpurun_out/prof_tl.log 2>&1
cd $R
python3 benchmarks/trace_gaps.py gpurun_out/prof_tl --steps 5 --out gpurun_out/gpt2_timeline.md
rm -rf gpurun_out/prof_tl
