set -e
# round 5: AdamW grid-size A/B (NBD_ADAMW_BLOCKS)
R=$GRAFT_REPO_ROOT
cd $R
for i in 1 2; do
  for b in 2048 1024 4096 8192 100000000; do
    echo "== blocks $b round $i"; NBD_ADAMW_BLOCKS=$b timeout -k 10 120 python benchmarks/ops_bench.py --only adamw
  done
done > gpurun_out/r5f_adamw_grid.txt 2>&1
# the notebook's HF-swap loop: whole step and host/GPU phases, with and without accelerate
timeout -k 10 180 python -u benchmarks/hfnative_loop.py --steps 30 --warm 8 --phases > gpurun_out/r5f_hfnative.txt 2>&1
timeout -k 10 180 python -u benchmarks/hfnative_loop.py --steps 30 --warm 8 --phases --no-accelerate >> gpurun_out/r5f_hfnative.txt 2>&1
# per-shape HIP vs hipBLASLt GEMMs
timeout -k 10 300 python -u benchmarks/gemm_bench.py --json gpurun_out/r5f_gemm.json > gpurun_out/r5f_gemm.txt 2>&1
# short-sequence attention: latency vs batch (pipelined GPU time per call)
timeout -k 10 120 python -u benchmarks/attn_bench.py --only smollm2_causal,b1,b4,b64,t256 --shape b1,1,9,3,128,1 --shape b4,4,9,3,128,1 --shape b64,64,9,3,128,1 --shape t256,16,9,3,256,1 > gpurun_out/r5f_attn_short.txt 2>&1
