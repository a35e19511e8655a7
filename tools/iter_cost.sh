#!/bin/bash
# Per-iteration counters of wave_kernel: two fixed-work runs (tools/iter_cost.py) per counter set.
set -uo pipefail
export TMPDIR=/tmp
OUT=${1:?outdir}
mkdir -p "$OUT"
S1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU"
S2="SQ_INSTS_MFMA SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC"
for it in 100 200; do
  for set in 1 2; do
    eval C=\$S$set
    timeout -s KILL 90 rocprofv3 --pmc $C --kernel-include-regex wave_kernel --output-format csv \
      -d "$OUT/i${it}_s$set" -o pmc -- python3 tools/iter_cost.py --iters $it > "$OUT/i${it}_s$set.out" 2>&1 || exit 1
  done
done
python3 - "$OUT" << 'PY'
import csv, glob, sys, collections
o = sys.argv[1]
def read(d):
    per = collections.defaultdict(dict)
    for fn in glob.glob(f"{o}/{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(fn)):
            per[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
    ks = sorted(per, key=int)[1:]  # drop the cold first dispatch
    agg = collections.defaultdict(float)
    for k in ks:
        for c, v in per[k].items():
            agg[c] += v / len(ks)
    return agg
B = 4096
for s in (1, 2):
    a, b = read(f"i100_s{s}"), read(f"i200_s{s}")
    for c in sorted(a):
        print(f"{c:24s} per-robot@100 {a[c]/B:12.1f}  per-iteration {(b[c]-a[c])/B/100:10.2f}")
PY
