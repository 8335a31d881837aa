set -e
# round 5: HF-swap loop with stack graphs on / off, and block graphs off (hoisted casts)
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONUNBUFFERED=1
for i in 1 2 3; do
  echo "== stacks on (default) round $i"; timeout -k 10 180 python -u benchmarks/hfnative_loop.py --steps 30 --warm 8 --phases
  echo "== stacks off round $i"; NBD_BLOCK_STACKS=0 timeout -k 10 180 python -u benchmarks/hfnative_loop.py --steps 30 --warm 8 --phases
  echo "== block graphs off round $i"; NBD_BLOCK_GRAPHS=0 timeout -k 10 180 python -u benchmarks/hfnative_loop.py --steps 30 --warm 8 --phases
done > gpurun_out/r5k_hfnative.txt 2>&1
