set -e
# round 5 (session 2): bench line with the graphed GPT-2 arm on the hand-written LM head
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u bench.py > gpurun_out/r5ab_bench.json 2> gpurun_out/r5ab_bench.log
