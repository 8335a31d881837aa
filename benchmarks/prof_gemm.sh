set -e
# rocprofv3 evidence for the HIP GEMM: PMC passes over gemm_bench (MFMA / LDS counters, HBM
# bytes) and kernel-trace breakdowns of the graphed GPT-2 and SmolLM2 training steps.
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $R/gpurun_out/pmcG_A -o pmc -- python3 $R/benchmarks/gemm_bench.py > $R/gpurun_out/pmcG_A.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/pmcG_B -o pmc -- python3 $R/benchmarks/gemm_bench.py > $R/gpurun_out/pmcG_B.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_gpt2g -o p -- python3 $R/benchmarks/ddp_compare.py --impls flatgraph --rounds 1 --steps 10 --warm 3 > $R/gpurun_out/prof_gpt2g.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_nbg -o p -- python3 $R/benchmarks/notebook_step.py --modes nbdgraph --steps 20 --warm 3 > $R/gpurun_out/prof_nbg.log 2>&1
cd $R
python3 benchmarks/pmc_summary.py gpurun_out/pmcG_A gpurun_out/pmcG_B --out gpurun_out/pmc_gemm.md > gpurun_out/pmc_gemm_summary.log 2>&1
python3 benchmarks/summarize_rocprof.py gpurun_out/prof_gpt2g gpurun_out/gpt2_graph_prof.md --title "GPT-2 small flat DDP step, HIP graph, HIP GEMM (13 replays incl. warm-up)" --top 40
python3 benchmarks/summarize_rocprof.py gpurun_out/prof_nbg gpurun_out/notebook_graph_prof.md --title "SmolLM2-135M-cls notebook step, HIP graph, HIP GEMM (23 replays incl. warm-up)" --top 40
rm -rf gpurun_out/pmcG_A gpurun_out/pmcG_B gpurun_out/prof_gpt2g gpurun_out/prof_nbg
