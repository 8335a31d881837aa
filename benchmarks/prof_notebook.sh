set -e
# kernel breakdown of the reference notebook's step on the native Llama path (graphed)
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_nb -o p -- python3 $R/benchmarks/notebook_step.py --modes nbdgraph --steps 20 --warm 3 > $R/gpurun_out/prof_nb.log 2>&1
cd $R
python3 benchmarks/summarize_rocprof.py gpurun_out/prof_nb gpurun_out/notebook_prof.md --title "SmolLM2-135M-cls native Llama step, HIP graph (23 replays + capture warm-up)" --top 40
rm -rf gpurun_out/prof_nb
