set -e
# round 5 (session 2): non-temporal C stores in gemm256 (variant 6) — tests, the LM-head products
# A/B, then the GPT-2 step with the library head and the hand-written one, interleaved
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm256.py tests/test_gpu_xent_fused.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5y_tests.txt 2>&1
timeout -k 10 400 python -u benchmarks/g256_ct_ab.py --rounds 3 --iters 10 --variants 4,6 --shapes lm > gpurun_out/r5y_ab.txt 2>&1
for r in 1 2 3; do
  for v in 0 1; do
    echo "== NBD_LMHEAD_HIP=$v round $r" >> gpurun_out/r5y_step.txt
    NBD_LMHEAD_HIP=$v timeout -k 10 200 python -u benchmarks/ddp_compare.py --impls flat,flatgraph --rounds 1 --steps 10 --warm 3 2>&1 | grep "ms/step" >> gpurun_out/r5y_step.txt
  done
done
