# round 5: the N = 2 bench paths on one GPU (both ranks on cuda:0, gloo: RCCL refuses two ranks on
# one device) — torchrun attach and self-launch; every arm either measures or records its error
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONUNBUFFERED=1 NBD_BENCH_HARD_S=420
timeout -k 10 480 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 5 --warmup 2 --backend gloo > gpurun_out/r5n_torchrun.json 2> gpurun_out/r5n_torchrun.log
rc=$?
echo "torchrun rc=$rc"
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 480 python bench.py --gpus 2 --steps 5 --warmup 2 --backend gloo > gpurun_out/r5n_self.json 2> gpurun_out/r5n_self.log
echo "self rc=$?"
