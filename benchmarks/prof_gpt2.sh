set -e
# rocprofv3 kernel breakdown of the GPT-2 small DDP step (flat bf16 + FlatAdamW, and amp for contrast)
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_gpt2_flat -o p -- python3 $R/benchmarks/ddp_compare.py --impls flat --rounds 1 --steps 10 --warm 3 > $R/gpurun_out/prof_gpt2_flat.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_gpt2_amp -o p -- python3 $R/benchmarks/ddp_compare.py --impls nbd --rounds 1 --steps 10 --warm 3 > $R/gpurun_out/prof_gpt2_amp.log 2>&1
cd $R
python3 benchmarks/summarize_rocprof.py gpurun_out/prof_gpt2_flat gpurun_out/gpt2_flat.md --title "GPT-2 small flat DDP step, 13 steps" --top 40
python3 benchmarks/summarize_rocprof.py gpurun_out/prof_gpt2_amp gpurun_out/gpt2_amp.md --title "GPT-2 small amp DDP step, 13 steps" --top 40
rm -rf gpurun_out/prof_gpt2_flat gpurun_out/prof_gpt2_amp
