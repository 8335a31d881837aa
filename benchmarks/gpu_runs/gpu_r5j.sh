set -e
# round 5: native() casts grouped across layers at world size 1 (one cast node), the stack's cast-epoch guard
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_swap_semantics.py tests/test_gpu_block_graphs.py tests/test_gpu_llama.py > gpurun_out/r5j_tests.log 2>&1
timeout -k 10 240 python -u benchmarks/native_bg_check.py --steps 10 > gpurun_out/r5j_bgcheck.txt 2>&1
for i in 1 2 3; do
  echo "== cast all layers (default) round $i"; timeout -k 10 180 python -u benchmarks/hfnative_loop.py --steps 30 --warm 8 --phases
  echo "== cast per layer round $i"; NBD_NATIVE_CAST_LAYERS=1 timeout -k 10 180 python -u benchmarks/hfnative_loop.py --steps 30 --warm 8 --phases
done > gpurun_out/r5j_hfnative.txt 2>&1
