set -e
# round 5 (session 2): gemm256 variant 7 (LM-head forward: C stores straight from the accumulators)
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm256.py > gpurun_out/r5as_tests.txt 2>&1
timeout -k 10 300 python -u benchmarks/gemm_tile_ab.py --shape 8192,50688,768 --hints 88256256,89256256,88256256,89256256 > gpurun_out/r5as_head.txt 2>&1
