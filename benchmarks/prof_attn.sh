set -e
# kernel breakdown of the GPT-2 flat DDP step + PMC counters of the attention kernels
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_gpt2_flat -o p -- python3 $R/benchmarks/ddp_compare.py --impls flat --rounds 1 --steps 10 --warm 3 > $R/gpurun_out/prof_gpt2_flat.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAIT_INST_LDS --kernel-trace --output-format csv -d $R/gpurun_out/pmcA -o pmc -- python3 $R/benchmarks/ops_bench.py --only attn > $R/gpurun_out/pmcA.log 2>&1
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmcB -o pmc -- python3 $R/benchmarks/ops_bench.py --only attn > $R/gpurun_out/pmcB.log 2>&1
cd $R
python3 benchmarks/summarize_rocprof.py gpurun_out/prof_gpt2_flat gpurun_out/gpt2_flat.md --title "GPT-2 small flat DDP step (HIP flash attention + fused CE), 13 steps" --top 40
python3 benchmarks/pmc_summary.py gpurun_out/pmcA gpurun_out/pmcB --out gpurun_out/pmc_attn.md --filter "attn|fwd|bwd" > gpurun_out/pmc_attn.log 2>&1
rm -rf gpurun_out/prof_gpt2_flat gpurun_out/pmcA gpurun_out/pmcB
