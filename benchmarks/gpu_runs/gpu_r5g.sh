set -e
# round 5: attention one-wave workgroups (short sequences), native() backward graphs through cast
# gradient destinations, AdamW without a grid cap, GEMMs vs hipBLASLt (pipelined, TunableOp)
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_swap_semantics.py tests/test_gpu_block_graphs.py tests/test_gpu_graddst.py tests/test_gpu_llama.py tests/test_gpu_attn.py > gpurun_out/r5g_tests.log 2>&1
SH="--only smollm2_causal,gpt2_causal,b1,b4,b64,t256 --shape b1,1,9,3,128,1 --shape b4,4,9,3,128,1 --shape b64,64,9,3,128,1 --shape t256,16,9,3,256,1"
for i in 1 2; do
  echo "== auto round $i"; timeout -k 10 120 python -u benchmarks/attn_bench.py $SH
  echo "== nw4 round $i"; NBD_ATTN_NW=4 timeout -k 10 120 python -u benchmarks/attn_bench.py $SH
  echo "== auto+gsplit1 round $i"; NBD_ATTN_GSPLIT=1 timeout -k 10 120 python -u benchmarks/attn_bench.py $SH
done > gpurun_out/r5g_attn_nw.txt 2>&1
for i in 1 2; do
  for g in 1 2; do
    echo "== native block_graphs $g round $i"
    NBD_NATIVE_BLOCK_GRAPHS=$g timeout -k 10 180 python -u benchmarks/hfnative_loop.py --steps 30 --warm 8 --phases
  done
done > gpurun_out/r5g_hfnative.txt 2>&1
timeout -k 10 120 python -u benchmarks/ops_bench.py --only adamw > gpurun_out/r5g_adamw.txt 2>&1
timeout -k 10 300 python -u benchmarks/gemm_bench.py --pipelined --json gpurun_out/r5g_gemm_pipe.json > gpurun_out/r5g_gemm_pipe.txt 2>&1
timeout -k 10 400 python -u benchmarks/gemm_bench.py --pipelined --tunableop --json gpurun_out/r5g_gemm_tuned.json > gpurun_out/r5g_gemm_tuned.txt 2>&1
