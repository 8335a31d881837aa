set -e
# round 5 (session 2): GPT-2 tied-table padding 512 vs 256 with the hand-written LM head
# (50688 vs 50432 rows: one 256-row tile column fewer, input-gradient split 8 vs 4), interleaved
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
for r in 1 2 3; do
  for v in 512 256; do
    echo "== pad $v round $r" >> gpurun_out/r5ao_ab.txt
    NBD_GPT2_VOCAB_PAD=$v timeout -k 10 200 python -u benchmarks/ddp_compare.py --impls flat,flatgraph --rounds 1 --steps 10 --warm 3 2>&1 | grep "ms/step" >> gpurun_out/r5ao_ab.txt
  done
done
