set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_attn.py tests/test_gpu_norm.py tests/test_gpu_llama_block.py > gpurun_out/t_r3q.txt 2>&1
echo tests-ok
bash benchmarks/ab_lib.sh gpurun_ab/libnbd_ops_base.so "python benchmarks/notebook_step.py --modes nbd,nbdgraph --steps 30" 3 > gpurun_out/nb_norm_ab_r3q.txt 2>&1
echo ab-ok
bash benchmarks/ab_lib.sh gpurun_ab/libnbd_ops_base.so "python benchmarks/ddp_compare.py --impls flat,flatgraph --rounds 2 --steps 10" 2 > gpurun_out/gpt2_norm_ab_r3q.txt 2>&1
echo done
