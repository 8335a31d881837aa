set -e
# round 5 (session 2): LM-head weight gradient as whole rounds + a split tail — tests, then the
# GPT-2 step with the library head and the hand-written one, interleaved
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_xent_fused.py tests/test_gpu_gemm.py tests/test_gpu_gemm256.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5aa_tests.txt 2>&1
for r in 1 2 3; do
  for v in 0 1; do
    echo "== NBD_LMHEAD_HIP=$v round $r" >> gpurun_out/r5aa_step.txt
    NBD_LMHEAD_HIP=$v timeout -k 10 200 python -u benchmarks/ddp_compare.py --impls flat,flatgraph --rounds 1 --steps 10 --warm 3 2>&1 | grep "ms/step" >> gpurun_out/r5aa_step.txt
  done
done
