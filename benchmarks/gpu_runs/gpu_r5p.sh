set -e
# round 5 (session 2): gemm256 contiguous-halves variants — tests, then the A/B against the banded
# halves, the 128x128 kernel and hipBLASLt (sq4096 / LM head / GPT-2 backward shapes)
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm256.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5p_tests.txt 2>&1
timeout -k 10 400 python -u benchmarks/g256_ct_ab.py --rounds 3 --iters 10 > gpurun_out/r5p_ab.txt 2>&1
