#!/usr/bin/env bash
# One parameterised GPU-call runner (replaces the per-call gpu_rNx.sh scripts of rounds 4-5, which
# remain in git history).  Run from the repo root on the GPU box, e.g.
#
#   gpurun --timeout 1100 -- 'bash benchmarks/gpu_runs/run.sh r6a tests tests/test_gpu_gemm.py \
#                             -- bench -- prof benchmarks/gemm_bench.py --pipelined'
#
#   run.sh TAG STEP [ARGS...] [-- STEP [ARGS...]] ...
#
# STEPs (each under its own time limit; the first failure ends the call — no GPU step runs after
# a fault, an abort or a time-out):
#   tests [FILES...]        pytest -m gpu (all GPU tests when no file is given)
#   smoke                   __graft_entry__.smoke()
#   bench [ARGS...]         python bench.py ARGS            -> gpurun_out/TAG_bench.json / .log
#   py SCRIPT [ARGS...]     python SCRIPT ARGS              -> gpurun_out/TAG_<script>.txt
#   prof SCRIPT [ARGS...]   rocprofv3 --kernel-trace --stats around SCRIPT -> gpurun_out/TAG_prof/
#   sh SCRIPT [ARGS...]     bash SCRIPT ARGS (e.g. benchmarks/prof_gpt2_graph.sh: profile + summary)
#   ab VAR V1,V2 ROUNDS SCRIPT [ARGS...]
#                           interleaved A/B: ROUNDS x (VAR=V1, VAR=V2, ...) python SCRIPT ARGS
#                           -> gpurun_out/TAG_ab_<VAR>.txt (cdna_hip_programming.md §5.4 rule 24)
# Step time limits: NBD_RUN_TESTS_S (900), NBD_RUN_STEP_S (600).
set -u -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
export TMPDIR=${TMPDIR:-/tmp}
TAG=$1
shift
TESTS_S=${NBD_RUN_TESTS_S:-900}
STEP_S=${NBD_RUN_STEP_S:-600}

run_step() {
  local kind=$1
  shift
  local base
  case "$kind" in
    tests)
      local files=("$@")
      [ ${#files[@]} -eq 0 ] && files=(tests)
      timeout -k 10 "$TESTS_S" python -u -m pytest "${files[@]}" -m gpu -x -v --timeout 200 \
        --timeout-method thread > "gpurun_out/${TAG}_tests.txt" 2>&1 ;;
    smoke)
      timeout -k 10 "$STEP_S" python -u -c "import __graft_entry__ as g; g.smoke()" > "gpurun_out/${TAG}_smoke.txt" 2>&1 ;;
    bench)
      timeout -k 10 "$STEP_S" python -u bench.py "$@" > "gpurun_out/${TAG}_bench.json" 2> "gpurun_out/${TAG}_bench.log" ;;
    py)
      base=$(basename "$1" .py)
      timeout -k 10 "$STEP_S" python -u "$@" > "gpurun_out/${TAG}_${base}.txt" 2>&1 ;;
    prof)
      base=$(basename "$1" .py)
      timeout -k 10 "$STEP_S" rocprofv3 --kernel-trace --stats -d "gpurun_out/${TAG}_prof" -o "$base" \
        -- python3 -u "$@" > "gpurun_out/${TAG}_prof_${base}.txt" 2>&1 ;;
    sh)
      base=$(basename "$1" .sh)
      timeout -k 10 "$STEP_S" bash "$@" > "gpurun_out/${TAG}_${base}.txt" 2>&1 ;;
    ab)
      local var=$1 vals=$2 rounds=$3
      shift 3
      local out="gpurun_out/${TAG}_ab_${var}.txt"
      for r in $(seq 1 "$rounds"); do
        for v in ${vals//,/ }; do
          echo "== $var=$v round $r" >> "$out"
          env "$var=$v" timeout -k 10 "$STEP_S" python -u "$@" >> "$out" 2>&1 || return $?
        done
      done ;;
    *)
      echo "run.sh: unknown step '$kind'" >&2
      return 2 ;;
  esac
}

args=()
while [ $# -gt 0 ]; do
  if [ "$1" = "--" ]; then
    run_step "${args[@]}" || { rc=$?; echo "run.sh: step '${args[0]}' failed ($rc)"; exit "$rc"; }
    args=()
  else
    args+=("$1")
  fi
  shift
done
if [ ${#args[@]} -gt 0 ]; then
  run_step "${args[@]}" || { rc=$?; echo "run.sh: step '${args[0]}' failed ($rc)"; exit "$rc"; }
fi
echo "run.sh: all steps done"
