# LDS-array cycles and bank conflicts of wave_kernel per ADMM iteration (two fixed-work runs)
set -uo pipefail
export TMPDIR=/tmp
OUT=${1:?outdir}
mkdir -p "$OUT"
C="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL"
for it in 100 200; do
  timeout -s KILL 90 rocprofv3 --pmc $C --kernel-include-regex wave_kernel --output-format csv \
    -d "$OUT/i${it}" -o pmc -- python3 tools/iter_cost.py --iters $it > "$OUT/i${it}.out" 2>&1 || exit 1
done
python3 - "$OUT" << 'PY'
import csv, glob, sys, collections
o = sys.argv[1]
def read(d):
    per = collections.defaultdict(dict)
    for fn in glob.glob(f"{o}/{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(fn)):
            per[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
    ks = sorted(per, key=int)[1:]
    agg = collections.defaultdict(float)
    for k in ks:
        for c, v in per[k].items():
            agg[c] += v / len(ks)
    return agg
a, b = read("i100"), read("i200")
for c in sorted(a):
    print(f"{c:26s} per-launch@100 {a[c]:14.1f}  per-robot-iteration {(b[c]-a[c])/100/4096:10.2f}")
PY
