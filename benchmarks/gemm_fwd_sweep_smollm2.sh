#!/bin/bash
# Forward tile sweep on the SmolLM2 notebook shapes (2048 tokens): q|k|v, o_proj, gate|up (+SwiGLU,
# epi 4), down.  Tile code = ks*10^8 + waves*10^7 + stages*10^6 + BM*1000 + BN.
set -e
for shape in "2048 960 576 0" "2048 576 576 0" "2048 3072 576 4" "2048 576 1536 0"; do
  set -- $shape
  for t in 2064064 3064064 202064064 203064064 2128064 3128064 2064128 3064128 202128064 202064128 2128096 3128096; do
    timeout -k 5 60 python benchmarks/gemm_one.py $1 $2 $3 --tile $t --epi $4 --iters 300 2>/dev/null || echo "$1x$2x$3 tile $t: n/a"
  done
done
