set -e
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $R/gpurun_out/pmcA -o pmc -- python3 $R/benchmarks/ops_bench.py --only summary,adamw,flatten,prereduce > $R/gpurun_out/pmcA.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/pmcB -o pmc -- python3 $R/benchmarks/ops_bench.py --only summary,adamw,flatten,prereduce > $R/gpurun_out/pmcB.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmcC -o pmc -- python3 $R/benchmarks/ops_bench.py --only summary,adamw,flatten,prereduce > $R/gpurun_out/pmcC.log 2>&1
cd $R
python3 benchmarks/pmc_summary.py gpurun_out/pmcA gpurun_out/pmcB gpurun_out/pmcC --out gpurun_out/pmc_ops.md > gpurun_out/pmc_summary.log 2>&1
rm -rf gpurun_out/pmcA gpurun_out/pmcB gpurun_out/pmcC
