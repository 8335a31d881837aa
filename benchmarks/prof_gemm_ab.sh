set -e
# A/B kernel breakdowns: HIP MFMA GEMM (NBD_HIP_GEMM=1) vs hipBLASLt (0) Linear layers, for the
# GPT-2 flat DDP step and the SmolLM2 notebook step (HIP graph)
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for g in 1 0; do
  export NBD_HIP_GEMM=$g
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_gpt2_$g -o p -- python3 $R/benchmarks/ddp_compare.py --impls flatgraph --rounds 1 --steps 10 --warm 3 > $R/gpurun_out/prof_gpt2_$g.log 2>&1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_nb_$g -o p -- python3 $R/benchmarks/notebook_step.py --modes nbdgraph --steps 20 --warm 3 > $R/gpurun_out/prof_nb_$g.log 2>&1
done
cd $R
for g in 1 0; do
  python3 benchmarks/summarize_rocprof.py gpurun_out/prof_gpt2_$g gpurun_out/gpt2_gemm$g.md --title "GPT-2 small flat DDP step (HIP graph), NBD_HIP_GEMM=$g" --top 45
  python3 benchmarks/summarize_rocprof.py gpurun_out/prof_nb_$g gpurun_out/nb_gemm$g.md --title "SmolLM2 notebook step (graph), NBD_HIP_GEMM=$g" --top 45
  rm -rf gpurun_out/prof_gpt2_$g gpurun_out/prof_nb_$g
done
