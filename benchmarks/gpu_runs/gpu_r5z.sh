set -e
# round 5 (session 2): kernel profiles of the graphed GPT-2 step, library LM head and hand-written
# LM head (NBD_LMHEAD_HIP=1: no library GEMM in the step)
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_g1 -o p -- python3 $R/benchmarks/ddp_compare.py --impls flatgraph --rounds 1 --steps 10 --warm 3 > $R/gpurun_out/r5z_g1.log 2>&1
NBD_LMHEAD_HIP=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_g2 -o p -- python3 $R/benchmarks/ddp_compare.py --impls flatgraph --rounds 1 --steps 10 --warm 3 > $R/gpurun_out/r5z_g2.log 2>&1
cd $R
python3 benchmarks/summarize_rocprof.py gpurun_out/prof_g1 gpurun_out/gpt2_graph_prof_r5s2.md --title "GPT-2 small flat DDP step, HIP graph, 13 replays (library LM head, round 5 end)" --top 60
python3 benchmarks/summarize_rocprof.py gpurun_out/prof_g2 gpurun_out/gpt2_graph_prof_lmhead_hip_r5.md --title "GPT-2 small flat DDP step, HIP graph, 13 replays, NBD_LMHEAD_HIP=1 (no library GEMM)" --top 60
rm -rf gpurun_out/prof_g1 gpurun_out/prof_g2
