set -e
# round 5: native() block_graphs 1 vs 2 numerics under AdamW; hfnative loop kernel profile; GQA split test
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_attn.py -k gqa > gpurun_out/r5h_tests.log 2>&1
timeout -k 10 240 python -u benchmarks/native_bg_check.py --steps 12 > gpurun_out/r5h_bgcheck.txt 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r5h_prof -o hfnative -- python3 benchmarks/hfnative_loop.py --steps 20 --warm 5 > gpurun_out/r5h_prof.log 2>&1
