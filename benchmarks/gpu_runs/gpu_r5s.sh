set -e
# round 5 (session 2): gemm256 with 32-bit DMA offsets (no K-loop spills in the transposed layouts) —
# tests, then the layout A/B against the 128x128 kernel and hipBLASLt; then the LM-head tests
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm256.py tests/test_gpu_xent_fused.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5s_tests.txt 2>&1
timeout -k 10 400 python -u benchmarks/g256_ct_ab.py --rounds 3 --iters 10 --variants 4,0,1 > gpurun_out/r5s_ab.txt 2>&1
