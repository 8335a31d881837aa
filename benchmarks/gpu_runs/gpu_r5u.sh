set -e
# round 5 (session 2): persistent gemm256 (variant 6) — tests, then the A/B on the LM-head / square /
# GPT-2 shapes
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm256.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5u_tests.txt 2>&1
timeout -k 10 400 python -u benchmarks/g256_ct_ab.py --rounds 3 --iters 10 --variants 4,6 > gpurun_out/r5u_ab.txt 2>&1
