set -e
# round 5: native() path — casts hoisted before the blocks (stack graphs read current weights),
# deferred reductions for the cast-weight gradients; tests; HF loop A/B; bench N=1
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_swap_semantics.py tests/test_gpu_block_graphs.py tests/test_gpu_graddst.py tests/test_gpu_llama.py tests/test_gpu_attn.py > gpurun_out/r5i_tests.log 2>&1
timeout -k 10 240 python -u benchmarks/native_bg_check.py --steps 12 > gpurun_out/r5i_bgcheck.txt 2>&1
for i in 1 2; do
  echo "== defer on (default) round $i"; timeout -k 10 180 python -u benchmarks/hfnative_loop.py --steps 30 --warm 8 --phases
  echo "== defer off round $i"; NBD_GRAD_DEFER=0 timeout -k 10 180 python -u benchmarks/hfnative_loop.py --steps 30 --warm 8 --phases
  echo "== block_graphs 2 round $i"; NBD_NATIVE_BLOCK_GRAPHS=2 timeout -k 10 180 python -u benchmarks/hfnative_loop.py --steps 30 --warm 8 --phases
done > gpurun_out/r5i_hfnative.txt 2>&1
timeout -k 10 560 python -u bench.py > gpurun_out/r5i_bench.json 2> gpurun_out/r5i_bench.log
