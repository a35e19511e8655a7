#!/bin/bash
# Round-2 (second half) evidence: full GPU test suite, default-path bench + rocprofv3 kernel
# stats, and the experimental path-5 bench.  usage: tools/evidence_r02b.sh OUTDIR
set -uo pipefail
export TMPDIR=/tmp
OUT=${1:?outdir}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.txt" 2>&1
rc=$?
tail -3 "$OUT/gpu_tests.txt"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run \
  -- python3 bench.py --steps 10 --warmup 2 --no-cpu > "$OUT/bench_under_rocprof.json" 2> "$OUT/rocprof.err" || exit $?
timeout -k 10 200 python3 bench.py --solver dx --steps 10 --warmup 2 --no-cpu > "$OUT/bench_dx.json" 2> "$OUT/bench_dx.err" || exit $?
timeout -k 10 200 python3 tools/dx_timing.py 3 5 > "$OUT/dx_timing.txt" 2>&1 || exit $?
python3 - "$OUT" << 'PY'
import csv, json, sys
o = sys.argv[1]
for f in ("bench.json", "bench_dx.json"):
    d = json.load(open(o + "/" + f))
    print(f, "value", round(d["value"]), "ms", round(d["ms_per_step"], 3), "frac", round(d["roofline"]["frac"], 4), "parity", d.get("parity"))
for r in csv.DictReader(open(o + "/trace/run_kernel_stats.csv")):
    print(r["Name"][:48], r["AverageNs"])
PY
cat "$OUT/dx_timing.txt" | grep path
