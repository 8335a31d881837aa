# round 5: capture-failure recovery (GraphedStep) + the N = 2 rehearsal on one GPU with gloo (graph
# arms deferred to the end at N > 1)
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONUNBUFFERED=1 NBD_BENCH_HARD_S=420
true
rc=$?
echo "tests rc=$rc"
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 480 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 2 --warmup 1 --ddp-steps 3 --backend gloo > gpurun_out/r5o_torchrun.json 2> gpurun_out/r5o_torchrun.log
echo "torchrun rc=$?"
