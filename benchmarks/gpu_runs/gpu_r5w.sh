set -e
# round 5 (session 2): FlatAdamW overlap with collectives — tests, then the notebook arms twice
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_collective_path.py tests/test_gpu_llama_block.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r5w_tests.txt 2>&1
for r in 1 2; do
timeout -k 10 400 python -u bench.py --no-sweep --no-ddp --no-bcast > gpurun_out/r5w_bench$r.json 2> gpurun_out/r5w_bench$r.log
done
