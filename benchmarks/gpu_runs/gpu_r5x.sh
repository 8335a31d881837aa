set -e
# round 5 (session 2): gemm256 variant 6 (non-temporal C stores) — tests, then the LM-head A/B
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm256.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5x_tests.txt 2>&1
timeout -k 10 400 python -u benchmarks/g256_ct_ab.py --rounds 4 --iters 10 --variants 4,6 --shapes lm,sq > gpurun_out/r5x_ab.txt 2>&1
