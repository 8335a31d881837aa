set -e
# round 5 (session 2): grouped-backward schedule sweep (pair_sched.py) on the current tree
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u benchmarks/pair_sched.py --rounds 3 --iters 20 > gpurun_out/r5ah_pair.txt 2>&1
