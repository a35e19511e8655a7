#!/bin/bash
# Round-5 GPU round trip (through gpurun from the repo root): the GPU tests with the accuracy
# sentinels logged, the bench line, rocprofv3 kernel stats of C2, and (with PMC=1) the N = 20
# MFMA-utilisation pass and the C2 / C4 HBM traffic passes.
#   usage: tools/r05_run.sh OUTDIR [PMC=1 in the environment]
set -euo pipefail
export TMPDIR=/tmp
OUT=${1:?outdir}
mkdir -p "$OUT"
export MPCQP_SENTINEL_LOG="$PWD/$OUT/sentinels.jsonl"
rm -f "$MPCQP_SENTINEL_LOG"
rc=0
timeout -k 10 400 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread \
  > "$OUT/gpu_tests.txt" 2>&1 || rc=$?
grep -E "^FAILED|passed|failed" "$OUT/gpu_tests.txt" | tail -12
# rc 1 = some tests failed (assertions): go on to the bench; anything else (a crash, abort, fault or
# time limit) ends the call here
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run \
  -- python3 bench.py --steps 10 --warmup 2 --no-cpu --no-extras > "$OUT/bench_under_rocprof.json" 2> "$OUT/rocprof.err"
if [ "${PMC:-0}" = 1 ]; then
  timeout -k 10 60 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
  mkdir -p "$OUT/n20"
  timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    --kernel-include-regex "wave_kernel" --output-format csv -d "$OUT/n20/pmc_mfma" -o pmc \
    -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-extras --horizon 20 > /dev/null 2> "$OUT/n20/rocprof_mfma.err"
  timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-include-regex "wave_kernel" --output-format csv \
    -d "$OUT/n20/pmc_grbm" -o pmc -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-extras --horizon 20 > /dev/null 2> "$OUT/n20/rocprof_grbm.err"
  for H in 10 20; do
    timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "scale_kernel|wave_kernel" --output-format csv \
      -d "$OUT/h$H/pmc/fetch" -o pmc -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-extras --horizon $H > /dev/null 2> "$OUT/h$H.fetch.err"
    timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "scale_kernel|wave_kernel" --output-format csv \
      -d "$OUT/h$H/pmc/write" -o pmc -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-extras --horizon $H > /dev/null 2> "$OUT/h$H.write.err"
  done
fi
python3 - "$OUT" << 'PY'
import csv, json, sys
o = sys.argv[1]
d = json.load(open(o + "/bench.json"))
print("value", round(d["value"]), "ms", round(d["ms_per_step"], 3), "frac", round(d["roofline"]["frac"], 4),
      "parity", d.get("parity"))
for k, v in (d.get("extras") or {}).items():
    if isinstance(v, dict) and "value" in v:
        print(" ", k, round(v["value"]), v.get("parity", {}).get("max_rel_err_u0") if isinstance(v.get("parity"), dict) else "")
for r in csv.DictReader(open(o + "/trace/run_kernel_stats.csv")):
    print(r["Name"][:60], r["Calls"], r["AverageNs"])
PY
python3 tools/trace_span.py "$OUT/trace/run_kernel_trace.csv" | tee "$OUT/trace_span.json"
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('bench under rocprof: kernel_ms', r['kernel_ms'], 'parts', r.get('parts'))" "$OUT/bench_under_rocprof.json"
if [ "${CONTENTION:-0}" = 1 ]; then
  bash tools/r05_contention.sh "$OUT/contention"
fi
if [ "${PMCSQ:-0}" = 1 ]; then
  mkdir -p "$OUT/sq"
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_IFETCH \
    --kernel-include-regex "wave_kernel" --output-format csv -d "$OUT/sq/p1" -o pmc \
    -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-extras > /dev/null 2> "$OUT/sq/p1.err"
fi
if [ "${MB:-0}" = 1 ]; then
  timeout -k 10 60 tools/mb/mb_valu > "$OUT/mb_valu.txt" 2>&1 && cat "$OUT/mb_valu.txt"
fi
