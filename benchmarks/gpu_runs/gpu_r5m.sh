set -e
# round 5: full GPU suite + smoke + bench N=1
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r5m_gputests.txt 2>&1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5m_smoke.txt 2>&1
timeout -k 10 560 python -u bench.py > gpurun_out/r5m_bench.json 2> gpurun_out/r5m_bench.log
