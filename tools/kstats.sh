#!/bin/bash
# rocprofv3 kernel-trace stats of a short bench run: usage tools/kstats.sh OUTDIR [bench args...]
set -euo pipefail
export TMPDIR=/tmp
OUT=${1:?outdir}
shift
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run \
  -- python3 bench.py --steps 10 --warmup 2 --no-cpu "$@" > "$OUT/bench_under_rocprof.json" 2> "$OUT/rocprof_trace.err"
