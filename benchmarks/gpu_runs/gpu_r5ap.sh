set -e
# round 5 (session 2): per-shape GEMM table (HIP vs hipBLASLt, back-to-back launches) and the
# attention bench on the final round-5 tree
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u benchmarks/gemm_bench.py --pipelined --json gpurun_out/r5ap_gemm.json > gpurun_out/r5ap_gemm.txt 2>&1
timeout -k 10 300 python -u benchmarks/attn_bench.py > gpurun_out/r5ap_attn.txt 2>&1
