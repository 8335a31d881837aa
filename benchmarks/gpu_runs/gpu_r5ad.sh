set -e
# round 5 (session 2): nbd::adamw_tensors for the one-line swap's AdamW — tests, then the HF-swap
# loop with torch's fused AdamW and with the HIP step, interleaved
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_swap_semantics.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r5ad_tests.txt 2>&1
for r in 1 2 3; do
  for v in 0 1; do
    echo "== NBD_NATIVE_NBD_ADAMW=$v round $r" >> gpurun_out/r5ad_loop.txt
    NBD_NATIVE_NBD_ADAMW=$v timeout -k 10 200 python -u benchmarks/hfnative_loop.py --steps 30 --warm 8 2>&1 | grep -v "amdgpu.ids\|socket.cpp\|RCCL\|HIP version\|ROCm version\|Hostname\|Librccl" >> gpurun_out/r5ad_loop.txt
  done
done
