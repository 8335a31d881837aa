set -e
# rocprofv3 kernel breakdown of ring attention (zigzag, 1 rank) vs one flash call at T = 16k
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_ring -o p -- python3 $R/benchmarks/ring_bench.py --T 16384 > $R/gpurun_out/prof_ring.log 2>&1
cd $R
python3 benchmarks/summarize_rocprof.py gpurun_out/prof_ring gpurun_out/ring_rocprof.md --title "ring attention (zigzag, 1 rank) + flash, T=16384, H=12, fwd+bwd x13 each" --top 30
rm -rf gpurun_out/prof_ring
