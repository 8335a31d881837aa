#!/bin/bash
# Attention occupancy sweep: extra dynamic LDS per workgroup caps the resident workgroups per CU
# (NBD_ATTN_FWD_LDS_PAD / NBD_ATTN_BWD_LDS_PAD), so the dispatcher balances the causal grid.
#   bash benchmarks/attn_occ_sweep.sh [fwdpad:bwdpad ...]
# static LDS: fwd 21.5 KB (pad 0 -> <=6 WG/CU by VGPRs, 20000 -> 3, 34000 -> 2, 62000 -> 1);
#             bwd 37.4 KB (pad 0 -> 4, 5000 -> 3, 20000 -> 2, 46000 -> 1)
set -e
pairs=${*:-"0:0 20000:5000 34000:20000 62000:46000 0:0"}
for pr in $pairs; do
  f=${pr%%:*}; b=${pr##*:}
  echo "== fwd pad $f bwd pad $b"
  NBD_ATTN_FWD_LDS_PAD=$f NBD_ATTN_BWD_LDS_PAD=$b timeout -k 10 120 python benchmarks/attn_bench.py --iters 30 | grep -v '^{'
done
