set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_norm.py tests/test_gpu_llama_block.py tests/test_gpu_llama.py > gpurun_out/t_r3t.txt 2>&1
echo tests-ok
ROUNDS=3 bash benchmarks/nb_env_sweep.sh NBD_LN_BWD_RPI1=0 NBD_LN_BWD_RPI1=1 > gpurun_out/nb_rpi_ab_r3t.txt 2>&1
echo done
