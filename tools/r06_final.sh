#!/bin/bash
# Round-6 final evidence: bench line, C3-rank RCCL rates, rocprofv3 kernel stats + trace span, and the
# PMC passes (HBM traffic: FETCH_SIZE / WRITE_SIZE; executed FP64: SQ_INSTS_VALU_*_F64) for C2 and C4.
#   usage: tools/r06_final.sh OUTDIR
set -euo pipefail
export TMPDIR=/tmp
OUT=${1:?outdir}
mkdir -p "$OUT"
timeout -k 10 300 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
timeout -k 10 200 python3 bench.py --gpus 1 --dist --batch 8192 --no-extras --no-cpu --steps 20 > "$OUT/dist.json" 2> "$OUT/dist.err"
timeout -k 10 200 python3 bench.py --gpus 1 --batch 8192 --no-extras --no-cpu --steps 20 > "$OUT/plain.json" 2> "$OUT/plain.err"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run \
  -- python3 bench.py --steps 10 --warmup 2 --no-cpu --no-extras > "$OUT/bench_under_rocprof.json" 2> "$OUT/rocprof.err"
python3 tools/trace_span.py "$OUT/trace/run_kernel_trace.csv" > "$OUT/trace_span.json"
for H in 10 20; do
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "scale_kernel|wave_kernel" --output-format csv \
    -d "$OUT/h$H/pmc/fetch" -o pmc -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-extras --horizon $H > /dev/null 2> "$OUT/h$H.fetch.err"
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "scale_kernel|wave_kernel" --output-format csv \
    -d "$OUT/h$H/pmc/write" -o pmc -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-extras --horizon $H > /dev/null 2> "$OUT/h$H.write.err"
  timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAVE_CYCLES \
    --kernel-include-regex "scale_kernel|wave_kernel" --output-format csv -d "$OUT/flops/h$H" -o pmc \
    -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-extras --horizon $H > /dev/null 2> "$OUT/h$H.flops.err"
done
python3 tools/pmc_traffic.py "$OUT/h10/pmc" --key N10_B4096_trot --parts 3 --out "$OUT/pmc_traffic.json"
python3 tools/pmc_traffic.py "$OUT/h20/pmc" --key N20_B4096_trot --parts 3 --out "$OUT/pmc_traffic.json"
python3 tools/pmc_flops.py "$OUT/flops/h10" --key N10_B4096_trot --parts 3 --out "$OUT/pmc_flops.json"
python3 tools/pmc_flops.py "$OUT/flops/h20" --key N20_B4096_trot --parts 3 --out "$OUT/pmc_flops.json"
python3 - "$OUT" << 'PY'
import csv, json, sys
o = sys.argv[1]
last = lambda fn: json.loads([l for l in open(fn) if l.startswith("{")][-1])
d = last(o + "/bench.json")
r = d["roofline"]
print("value", round(d["value"]), "ms", round(d["ms_per_step"], 4), "frac", round(r["frac"], 4), "exec_frac", r.get("executed_frac"),
      "parity", d.get("parity"))
for k, v in (d.get("extras") or {}).items():
    if isinstance(v, dict) and "value" in v:
        print(" ", k, round(v["value"]))
a, b = last(o + "/dist.json"), last(o + "/plain.json")
print(f"rccl world 1 (one part): {a['value']:.0f} plain {b['value']:.0f} ratio {a['value'] / b['value']:.3f} allgather_ms {a['extras']['allgather_ms']}")
for rr in csv.DictReader(open(o + "/trace/run_kernel_stats.csv")):
    print(rr["Name"][:60], rr["Calls"], rr["AverageNs"])
print(open(o + "/trace_span.json").read())
PY
