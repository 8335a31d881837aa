# round 5 (session 2): the N = 2 bench on one GPU (gloo; both ranks on cuda:0) with the hand-written
# LM head default and the library-head arm — self-launched; every arm measures or records its error
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONUNBUFFERED=1 NBD_BENCH_HARD_S=560
timeout -k 10 600 python bench.py --gpus 2 --steps 3 --warmup 1 --ddp-steps 3 --backend gloo --no-notebook > gpurun_out/r5af_self.json 2> gpurun_out/r5af_self.log
echo "self rc=$?"
