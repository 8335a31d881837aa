set -e
# round 5: which hipBLASLt kernels beat the HIP GEMM on GPT-2's forward shapes; HIP tile sweep there
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r5l_lib -o lib -- python3 benchmarks/lib_gemm_probe.py > gpurun_out/r5l_lib.log 2>&1
timeout -k 10 400 python -u benchmarks/gemm_bench.py --pipelined --sweep > gpurun_out/r5l_sweep.txt 2>&1
