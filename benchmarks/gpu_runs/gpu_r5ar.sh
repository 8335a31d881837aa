set -e
# round 5 (session 2): the LM-head forward product (8192 x 50688 x 768) on every forward kernel
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u benchmarks/gemm_tile_ab.py --shape 8192,50688,768 --hints 88256256,86256256,82128128,83128128,2128096,82128192,83128192 > gpurun_out/r5ar_head.txt 2>&1
