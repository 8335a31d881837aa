#!/bin/bash
# Interleaved A/B of two builds: the tree in ./abtree_old (a git worktree of an earlier commit,
# built in place) against this tree.  bash benchmarks/gpu_runs/abtree.sh TAG ROUNDS SCRIPT [ARGS...]
# -> gpurun_out/TAG_abtree.txt.  Each run under its own time limit; the first failure ends it.
set -u -o pipefail
TAG=$1 ROUNDS=$2
shift 2
ROOT=$(pwd)
OUT="$ROOT/gpurun_out/${TAG}_abtree.txt"
mkdir -p "$ROOT/gpurun_out"
: > "$OUT"
for r in $(seq 1 "$ROUNDS"); do
  for side in old new; do
    echo "== $side round $r" >> "$OUT"
    if [ "$side" = old ]; then dir="$ROOT/abtree_old"; else dir="$ROOT"; fi
    (cd "$dir" && timeout -k 10 "${NBD_RUN_STEP_S:-600}" python -u "$@") >> "$OUT" 2>&1 || { echo "failed: $side round $r" >> "$OUT"; exit 1; }
  done
done
echo "abtree: all rounds done"
