set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_llama_block.py tests/test_gpu_llama.py tests/test_gpu_graddst.py > gpurun_out/t_r3w.txt 2>&1
echo tests-ok
ROUNDS=4 bash benchmarks/nb_env_sweep.sh NBD_FUSED_STACK=0 NBD_FUSED_STACK=1 > gpurun_out/nb_stack_ab_r3w.txt 2>&1
NBD_FUSED_STACK=0 timeout -k 10 200 python benchmarks/host_profile.py --model smollm2 --steps 5 > gpurun_out/host_stack0_r3w.txt 2>&1
timeout -k 10 200 python benchmarks/host_profile.py --model smollm2 --steps 5 > gpurun_out/host_stack1_r3w.txt 2>&1
echo done
