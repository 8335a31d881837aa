set -e
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 250 python bench.py > gpurun_out/diag_warm1_$i.json 2>/dev/null
  NBD_GEMM_WARM=0 timeout -k 10 250 python bench.py > gpurun_out/diag_warm0_$i.json 2>/dev/null
done
echo done
