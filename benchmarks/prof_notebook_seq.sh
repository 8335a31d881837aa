set -e
# kernel sequence of one graphed notebook step (benchmarks/trace_sequence.py over a kernel trace)
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_nb_seq -o p -- python3 $R/benchmarks/notebook_step.py --modes nbdgraph --steps 6 --warm 3 > $R/gpurun_out/prof_nb_seq.log 2>&1
cd $R
python3 benchmarks/trace_sequence.py gpurun_out/prof_nb_seq --last ${SEQ_LAST:-1100} --full > gpurun_out/nb_seq.txt
rm -rf gpurun_out/prof_nb_seq
