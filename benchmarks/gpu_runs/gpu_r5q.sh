set -e
# round 5 (session 2): kernel sequence of one graphed GPT-2 step and one graphed notebook step —
# where the copies, fills and torch elementwise kernels sit
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_g -o p -- python3 $R/benchmarks/ddp_compare.py --impls flatgraph --rounds 1 --steps 6 --warm 3 > $R/gpurun_out/r5q_g.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_n -o p -- python3 $R/benchmarks/notebook_step.py --modes nbdgraph --steps 6 --warm 3 > $R/gpurun_out/r5q_n.log 2>&1
cd $R
python3 benchmarks/trace_seq.py gpurun_out/prof_g --all > gpurun_out/r5q_gpt2_seq.txt
python3 benchmarks/trace_seq.py gpurun_out/prof_n --all > gpurun_out/r5q_nb_seq.txt
rm -rf gpurun_out/prof_g gpurun_out/prof_n
