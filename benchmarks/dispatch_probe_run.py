"""Run benchmarks/bin/dispatch_probe (benchmarks/dispatch_probe.hip) and summarise which blocks
share a CU: the placement the causal attention forward's block order is tuned for (FINDINGS §36).

    hipcc --offload-arch=gfx950 -O2 -o benchmarks/bin/dispatch_probe benchmarks/dispatch_probe.hip
    python benchmarks/dispatch_probe_run.py [grid per_cu spin_us] ...
"""
import collections
import subprocess
import sys
from pathlib import Path

BIN = Path(__file__).resolve().parent / "bin" / "dispatch_probe"


def run(grid: int, per_cu: int, spin_us: float):
    out = subprocess.run([str(BIN), str(grid), str(per_cu), str(spin_us)], check=True, capture_output=True,
                         text=True, timeout=60).stdout
    rows = [list(map(float, ln.split(","))) for ln in out.strip().splitlines()[1:]]
    cus = collections.defaultdict(list)
    for b, xcc, se, cu, t0, t1 in rows:
        cus[(int(xcc), int(se), int(cu))].append((int(b), t0, t1))
    print(f"== grid {grid}, {per_cu}/CU, spin {spin_us} us: {len(cus)} CUs used; "
          f"blocks/CU {collections.Counter(len(v) for v in cus.values())}")
    # block -> xcc map: is it b % 8?
    xcc_of = {int(r[0]): int(r[1]) for r in rows}
    lab = collections.defaultdict(set)
    for b, x in xcc_of.items():
        lab[b % 8].add(x)
    print("  b%8 -> xcc sets:", {k: sorted(v) for k, v in sorted(lab.items())})
    # within one CU: the block indices and their differences
    diffs = collections.Counter()
    shown = 0
    for key, v in sorted(cus.items()):
        bs = sorted(b for b, _, _ in v)
        diffs[tuple(bs[i + 1] - bs[i] for i in range(len(bs) - 1))] += 1
        if shown < 12:
            print(f"  cu {key}: blocks {bs} starts(us) {[round(t0 / 1e3, 2) for _, t0, _ in sorted(v)]}")
            shown += 1
    print("  gaps between a CU's blocks (most common):", diffs.most_common(8))
    starts = sorted(r[4] for r in rows)
    print(f"  start spread: first {starts[0] / 1e3:.2f} us, last {starts[-1] / 1e3:.2f} us")
    sys.stdout.flush()


def main(argv):
    cases = [(768, 3, 30.0), (1536, 6, 30.0), (512, 2, 30.0), (1152, 3, 30.0)]
    if argv:
        cases = [(int(argv[i]), int(argv[i + 1]), float(argv[i + 2])) for i in range(0, len(argv), 3)]
    for c in cases:
        run(*c)


if __name__ == "__main__":
    main(sys.argv[1:])
