set -e
# round 5: AdamW kernel variants A/B (NBD_ADAMW_VARIANT) + correctness under each
R=$GRAFT_REPO_ROOT
cd $R
for v in 1 2 3; do
  NBD_ADAMW_VARIANT=$v timeout -k 10 200 python -u -m pytest tests/test_gpu_ops.py -x -q -k "adamw" --timeout 120 --timeout-method thread > gpurun_out/r5e_adamw_tests_$v.log 2>&1
done
for i in 1 2 3; do
  for v in 0 1 2 3; do
    echo "== variant $v round $i"; NBD_ADAMW_VARIANT=$v timeout -k 10 120 python benchmarks/ops_bench.py --only adamw
  done
done > gpurun_out/r5e_adamw.txt 2>&1
