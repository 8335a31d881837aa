set -e
# round 5 (session 2): the hand-written LM head (NBD_LMHEAD_HIP=1, gemm256 after the spill fix) — numerics tests, then the graphed
# GPT-2 step with the library head and with the hand-written one, interleaved
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_xent_fused.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5t_tests.txt 2>&1
for r in 1 2; do
  for v in 0 1; do
    echo "== NBD_LMHEAD_HIP=$v round $r" >> gpurun_out/r5t_ab.txt
    NBD_LMHEAD_HIP=$v timeout -k 10 200 python -u benchmarks/ddp_compare.py --impls flat,flatgraph --rounds 1 --steps 10 --warm 3 2>&1 | grep -v "amdgpu.ids\|socket.cpp" >> gpurun_out/r5t_ab.txt
  done
done
