set -e
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python3 $R/benchmarks/notebook_step.py --modes fp32,bf16flat > $R/gpurun_out/notebook_step.txt 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_nb -o p -- python3 $R/benchmarks/notebook_step.py --modes bf16flat --steps 10 --warm 3 > $R/gpurun_out/prof_nb.log 2>&1
cd $R
python3 benchmarks/summarize_rocprof.py gpurun_out/prof_nb gpurun_out/notebook_prof.md --title "SmolLM2-135M-cls bf16flat step (13 steps)" --top 30
rm -rf gpurun_out/prof_nb
