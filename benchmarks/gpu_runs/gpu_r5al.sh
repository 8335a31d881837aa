set -e
# round 5 (session 2): GPT-2 step with the mlp.c_proj forward on the 128x192 tile vs 128x96
# (the tuned-table entry patched back for the base arm), interleaved; plus the tile's GPU tests
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py -k "128x96" > gpurun_out/r5al_tests.txt 2>&1
for r in 1 2 3; do
  for v in base t192; do
    echo "== $v round $r" >> gpurun_out/r5al_ab.txt
    timeout -k 10 200 python -u -c "
import runpy, sys
sys.argv = ['ddp_compare.py', '--impls', 'flatgraph', '--rounds', '1', '--steps', '10', '--warm', '3']
from nbdistributed_amd.ops import gemm as G
if '$v' == 'base':
    G._TUNED[(False, False, 8192, 768, 3072)] = (2128096, 1)
runpy.run_path('benchmarks/ddp_compare.py', run_name='__main__')
" 2>&1 | grep "ms/step" >> gpurun_out/r5al_ab.txt
  done
done
