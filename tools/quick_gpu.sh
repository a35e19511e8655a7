#!/bin/bash
# One GPU round trip for kernel iteration: GPU tests, bench line, rocprofv3 kernel stats.
#   tools/quick_gpu.sh OUTDIR [bench args...]
set -uo pipefail
export TMPDIR=/tmp
OUT=${1:?outdir}
shift
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.txt" 2>&1
rc=$?
tail -3 "$OUT/gpu_tests.txt"
[ $rc -eq 0 ] || exit $rc
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
