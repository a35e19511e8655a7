#!/bin/bash
# One GPU round trip while iterating on a kernel: GPU tests (failures reported, not fatal), then —
# unless the tests crashed or timed out — the bench line and rocprofv3 kernel stats.
#   tools/gpu_try.sh OUTDIR [bench args...]
set -uo pipefail
export TMPDIR=/tmp
OUT=${1:?outdir}
shift
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests -m gpu -q --maxfail=20 --timeout 120 --timeout-method thread > "$OUT/gpu_tests.txt" 2>&1
rc=$?
tail -25 "$OUT/gpu_tests.txt"
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 200 python bench.py "$@" > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run \
  -- python3 bench.py --steps 10 --warmup 2 --no-cpu --no-extras "$@" > "$OUT/bench_under_rocprof.json" 2> "$OUT/rocprof.err" || exit $?
python3 - "$OUT" << 'PY'
import csv, json, sys
o = sys.argv[1]
d = json.load(open(o + "/bench.json"))
print("value", round(d["value"]), "ms", round(d["ms_per_step"], 3), "parity", d.get("parity"), "iters", d["stats"]["mean_iters"])
for r in csv.DictReader(open(o + "/trace/run_kernel_stats.csv")):
    print(r["Name"][:48], r["AverageNs"])
PY
