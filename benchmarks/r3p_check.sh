set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_norm.py tests/test_gpu_ops.py tests/test_gpu_graddst.py tests/test_gpu_llama_block.py > gpurun_out/t_r3s.txt 2>&1
echo tests-ok
bash benchmarks/ab_lib.sh gpurun_ab/libnbd_ops_base.so "python benchmarks/embed_bench.py" 2 > gpurun_out/embed_ab_r3s.txt 2>&1
bash benchmarks/ab_lib.sh gpurun_ab/libnbd_ops_base.so "python benchmarks/notebook_step.py --modes nbd,nbdgraph --steps 30" 3 > gpurun_out/nb_embed_ab_r3s.txt 2>&1
echo ab-ok
bash benchmarks/ab_lib.sh gpurun_ab/libnbd_ops_base.so "python benchmarks/ddp_compare.py --impls flat,flatgraph --rounds 2 --steps 10" 2 > gpurun_out/gpt2_embed_ab_r3s.txt 2>&1
echo done
