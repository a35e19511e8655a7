#!/bin/bash
# scale_kernel threads-per-column A/B at one horizon: kernel stats + bench parity per variant library
#   tools/ab_scale_tpc.sh OUTDIR HORIZON lib1.so lib2.so ...
set -uo pipefail
export TMPDIR=/tmp
OUT=${1:?out}; N=${2:?horizon}; shift 2
mkdir -p "$OUT"
for L in "$@"; do
  b=$(basename "$L" .so)
  MPCQP_LIB="$L" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$b" -o run \
    -- python3 bench.py --horizon "$N" --steps 5 --warmup 2 --no-cpu --no-extras > "$OUT/$b.json" 2> "$OUT/$b.err" || exit $?
  python3 - "$OUT" "$b" << 'PY'
import csv, json, sys
o, b = sys.argv[1], sys.argv[2]
d = json.load(open(f"{o}/{b}.json"))
ks = {r["Name"].split("(")[0].split("::")[-1]: float(r["AverageNs"]) / 1e3 for r in csv.DictReader(open(f"{o}/{b}/run_kernel_stats.csv"))}
pa = d.get("parity") or {}
print(b, "QP/s", round(d["value"]), "parity", pa.get("iters_equal_frac"), pa.get("max_rel_err_u0"), {k: round(v, 1) for k, v in ks.items() if "kernel" in k})
PY
done
