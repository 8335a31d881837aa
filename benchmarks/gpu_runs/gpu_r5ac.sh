set -e
# round 5 (session 2): hand-written LM head with the LM-head table warmed into the MALL by the
# preceding HIP GEMM launch (NBD_LM_HEAD_WARM_MB), interleaved
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONUNBUFFERED=1 NBD_LMHEAD_HIP=1
for r in 1 2 3; do
  for w in 0 96 192; do
    echo "== NBD_LM_HEAD_WARM_MB=$w round $r" >> gpurun_out/r5ac_step.txt
    NBD_LM_HEAD_WARM_MB=$w timeout -k 10 200 python -u benchmarks/ddp_compare.py --impls flat,flatgraph --rounds 1 --steps 10 --warm 3 2>&1 | grep "ms/step" >> gpurun_out/r5ac_step.txt
  done
done
