set -e
# round 5: paired causal attention backward A/B + correctness, new seqcls_prep kernel
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 200 python -u -m pytest tests/test_gpu_swap_semantics.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5d_swap.log 2>&1
NBD_ATTN_PAIR=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_attn.py tests/test_gpu_llama.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5d_attn_tests.log 2>&1
for i in 1 2; do
  echo "== pair 0 round $i"; NBD_ATTN_PAIR=0 timeout -k 10 120 python benchmarks/attn_bench.py --only gpt2_causal,long4k_causal
  echo "== pair 1 round $i"; NBD_ATTN_PAIR=1 timeout -k 10 120 python benchmarks/attn_bench.py --only gpt2_causal,long4k_causal
done > gpurun_out/r5d_attn_pair.txt 2>&1
