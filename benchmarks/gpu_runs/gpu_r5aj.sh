set -e
# round 5 (session 2): non-temporal stores for the weight gradients (K-major-A epilogue, the split-K
# reduce of weight gradients, the deferred multi-split-K) — A/B against the previous build (NBD_OPS_LIB), interleaved
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONUNBUFFERED=1
BASE=$R/nbdistributed_amd/_native/ab_base.so
for r in 1 2 3; do
  for v in base nt; do
    if [ $v = base ]; then export NBD_OPS_LIB=$BASE; else unset NBD_OPS_LIB; fi
    echo "== $v round $r" >> gpurun_out/r5aj_ab.txt
    timeout -k 10 200 python -u benchmarks/ddp_compare.py --impls flatgraph --rounds 1 --steps 10 --warm 3 2>&1 | grep "ms/step" >> gpurun_out/r5aj_ab.txt
    timeout -k 10 200 python -u benchmarks/notebook_step.py --modes nbdgraph --steps 20 --warm 5 2>&1 | grep -i "ms" | grep -v "amdgpu\|socket" >> gpurun_out/r5aj_ab.txt
  done
done
