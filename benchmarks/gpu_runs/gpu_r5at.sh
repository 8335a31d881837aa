set -e
# round 5 (session 2): the final in-tree build — full GPU suite and smoke
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r5at_gputests.txt 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5at_smoke.txt 2>&1
