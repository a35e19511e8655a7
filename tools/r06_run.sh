#!/bin/bash
# Round-6 GPU round trip (through gpurun from the repo root): the GPU tests with the accuracy
# sentinels logged, a bitwise A/B of the product library against exp/BASE.so (when given), the bench
# line, the C3-rank RCCL rates with the split on / off, and rocprofv3 kernel stats of C2.
#   usage: tools/r06_run.sh OUTDIR [BASE]
set -euo pipefail
export TMPDIR=/tmp
OUT=${1:?outdir}
BASE=${2:-}
mkdir -p "$OUT"
export MPCQP_SENTINEL_LOG="$PWD/$OUT/sentinels.jsonl"
rm -f "$MPCQP_SENTINEL_LOG"
rc=0
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread \
  > "$OUT/gpu_tests.txt" 2>&1 || rc=$?
grep -E "^FAILED|passed|failed" "$OUT/gpu_tests.txt" | tail -12
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
if [ -n "$BASE" ]; then
  timeout -k 10 200 python3 tools/ab_bitwise.py dump "$OUT/ab_new.npz" > "$OUT/ab.txt" 2>&1
  MPCQP_LIB=$PWD/exp/$BASE.so timeout -k 10 200 python3 tools/ab_bitwise.py dump "$OUT/ab_base.npz" >> "$OUT/ab.txt" 2>&1
  python3 tools/ab_bitwise.py cmp "$OUT/ab_base.npz" "$OUT/ab_new.npz" >> "$OUT/ab.txt" || true; tail -3 "$OUT/ab.txt"
  rm -f "$OUT"/ab_*.npz
fi
timeout -k 10 300 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
for SP in 0 1; do
  MPCQP_SPLIT=$SP timeout -k 10 200 python3 bench.py --gpus 1 --dist --batch 8192 --no-extras --no-cpu --steps 20 \
    > "$OUT/dist_split$SP.json" 2> "$OUT/dist_split$SP.err"
  MPCQP_SPLIT=$SP timeout -k 10 200 python3 bench.py --gpus 1 --batch 8192 --no-extras --no-cpu --steps 20 \
    > "$OUT/plain_split$SP.json" 2> "$OUT/plain_split$SP.err"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run \
  -- python3 bench.py --steps 10 --warmup 2 --no-cpu --no-extras > "$OUT/bench_under_rocprof.json" 2> "$OUT/rocprof.err"
python3 - "$OUT" << 'PY'
import csv, json, sys
o = sys.argv[1]
d = json.load(open(o + "/bench.json"))
print("value", round(d["value"]), "ms", round(d["ms_per_step"], 4), "frac", round(d["roofline"]["frac"], 4),
      "parity", d.get("parity"))
for k, v in (d.get("extras") or {}).items():
    if isinstance(v, dict) and "value" in v:
        print(" ", k, round(v["value"]))
def last(fn):
    return json.loads([l for l in open(fn) if l.startswith("{")][-1])
for sp in (0, 1):
    a = last(f"{o}/dist_split{sp}.json"); b = last(f"{o}/plain_split{sp}.json")
    print(f"split={sp} (0 = auto): dist {a['value']:.0f} plain {b['value']:.0f} ratio {a['value'] / b['value']:.3f} allgather_ms {a['extras']['allgather_ms']}")
for r in csv.DictReader(open(o + "/trace/run_kernel_stats.csv")):
    print(r["Name"][:60], r["Calls"], r["AverageNs"])
PY
python3 tools/trace_span.py "$OUT/trace/run_kernel_trace.csv" | tee "$OUT/trace_span.json"
