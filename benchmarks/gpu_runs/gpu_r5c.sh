set -e
# round 5: swap-semantics GPU tests, K3 no_sync timing, notebook + GPT-2 graphed kernel profiles
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_swap_semantics.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r5c_swap.log 2>&1
timeout -k 10 200 python benchmarks/ops_bench.py --only prereduce > gpurun_out/r5c_k3.txt 2>&1
timeout -k 10 200 python benchmarks/attn_bench.py > gpurun_out/r5c_attn.txt 2>&1
bash benchmarks/prof_notebook.sh
bash benchmarks/prof_gpt2_graph.sh
