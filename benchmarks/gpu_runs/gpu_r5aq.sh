set -e
# round 5 (session 2) final: kernel profiles of the graphed GPT-2 step (hand-written LM head, the
# default) and the graphed notebook step on the final tree
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_g3 -o p -- python3 $R/benchmarks/ddp_compare.py --impls flatgraph --rounds 1 --steps 10 --warm 3 > $R/gpurun_out/r5aq_g3.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_nb3 -o p -- python3 $R/benchmarks/notebook_step.py --modes nbdgraph --steps 20 --warm 5 > $R/gpurun_out/r5aq_nb3.log 2>&1
cd $R
python3 benchmarks/summarize_rocprof.py gpurun_out/prof_g3 gpurun_out/gpt2_graph_prof_r5final.md --title "GPT-2 small flat DDP step, HIP graph, 13 replays (hand-written LM head, round 5 final tree)" --top 60
python3 benchmarks/summarize_rocprof.py gpurun_out/prof_nb3 gpurun_out/notebook_graph_prof_r5final2.md --title "SmolLM2-135M-cls native Llama step, HIP graph (round 5 final tree)" --top 40
rm -rf gpurun_out/prof_g3 gpurun_out/prof_nb3
