set -e
# round 5 (session 2): 128x192 8-wave forward tile vs the tuned kernels and hipBLASLt
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 200 python -u benchmarks/gemm_tile_ab.py --hints 82128192,83128192,82128128,2128096 > gpurun_out/r5ak_tile.txt 2>&1
timeout -k 10 200 python -u benchmarks/gemm_tile_ab.py --gelu --hints 82128192,83128192,82128128 >> gpurun_out/r5ak_tile.txt 2>&1
