set -e
# (the NBD_ATTN_FWD_ORDER knob existed only for this experiment and has been removed: docs/FINDINGS.md §16)
# forward causal block-order experiment (GPT-2 shape, 8 query blocks): NBD_ATTN_FWD_ORDER
for o in "" "7,6,5,4,3,2,1,0" "0,1,2,3,4,5,6,7" "7,0,6,1,5,2,4,3" "0,1,2,4,5,7,6,3" "3,4,2,5,1,6,0,7" ""; do
  echo "order=[$o] $(NBD_ATTN_FWD_ORDER=$o timeout -k 5 100 python benchmarks/attn_bench.py --iters 100 2>&1 | grep gpt2_causal)"
done
