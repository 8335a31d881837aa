set -e
# round 5 (session 2): full GPU suite + smoke + bench N=1 on the current tree
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r5v_gputests.txt 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5v_smoke.txt 2>&1
timeout -k 10 560 python -u bench.py > gpurun_out/r5v_bench.json 2> gpurun_out/r5v_bench.log
