set -e
# rocprofv3 kernel breakdown of the GPT-2 small flat DDP step
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_gpt2_graph -o p -- python3 $R/benchmarks/ddp_compare.py --impls flatgraph --rounds 1 --steps 10 --warm 3 > $R/gpurun_out/prof_gpt2_graph.log 2>&1
cd $R
python3 benchmarks/summarize_rocprof.py gpurun_out/prof_gpt2_graph gpurun_out/gpt2_graph_now.md --title "GPT-2 small flat DDP step, HIP graph, 13 replays (current tree)" --top 60
rm -rf gpurun_out/prof_gpt2_graph
