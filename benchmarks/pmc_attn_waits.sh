set -e
# rocprofv3 wave-state counters of the flash-attention kernels on one shape (ATTN_SHAPE, default
# the GPT-2 causal one): where their waves spend their cycles
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
SHAPE=${ATTN_SHAPE:-gpt2_causal}
timeout -k 10 -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS --kernel-trace --output-format csv -d $R/gpurun_out/pmcW -o pmc -- python3 $R/benchmarks/attn_bench.py --iters 20 --only $SHAPE > $R/gpurun_out/pmcW.log 2>&1
timeout -k 10 -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAVES --kernel-trace --output-format csv -d $R/gpurun_out/pmcX -o pmc -- python3 $R/benchmarks/attn_bench.py --iters 20 --only $SHAPE > $R/gpurun_out/pmcX.log 2>&1
cd $R
python3 - <<'PY'
import csv, glob, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float)); cnt = collections.Counter()
for d in ("gpurun_out/pmcW", "gpurun_out/pmcX"):
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "attn" not in k:
                continue
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
            if r["Counter_Name"] == "SQ_WAVES":
                cnt[k] += 1
for k, c in acc.items():
    n = max(cnt[k], 1)
    print(k[:90], "dispatches", n)
    for name, v in sorted(c.items()):
        print(f"  {name:28s} {v / n:14.4g}")
    wc = c.get("SQ_WAVE_CYCLES", 0)
    if wc:
        print(f"  wait_any {c['SQ_WAIT_ANY'] / wc:.3f}  wait_inst_any {c['SQ_WAIT_INST_ANY'] / wc:.3f}  active_inst {c['SQ_ACTIVE_INST_ANY'] / wc:.3f}  wait_inst_lds {c['SQ_WAIT_INST_LDS'] / wc:.3f}")
    if c.get("GRBM_GUI_ACTIVE"):
        print(f"  mfma_busy/simd-cycle {c['SQ_VALU_MFMA_BUSY_CYCLES'] / (1024 * c['GRBM_GUI_ACTIVE'] / 8):.3f}  lds_conflict/inst {c['SQ_LDS_BANK_CONFLICT'] / max(c['SQ_INSTS_LDS'], 1):.3f}")
PY
grep -h "fwd_us" gpurun_out/pmcW.log gpurun_out/pmcX.log
rm -rf gpurun_out/pmcW gpurun_out/pmcX
