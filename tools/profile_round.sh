#!/bin/bash
# GPU-box evidence pass for the default solve path (run through gpurun from the repo root):
# GPU tests, bench line, rocprofv3 kernel-trace stats of the bench, separate FETCH_SIZE /
# WRITE_SIZE counter passes over both solve kernels (TCC cannot hold both in one pass), the
# per-iteration SQ counters (tools/iter_cost.sh).  Each step has its own limit; the chain stops
# at the first failure.
#   usage: tools/profile_round.sh OUTDIR [bench args...]
set -euo pipefail
export TMPDIR=/tmp
OUT=${1:?outdir}
shift
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.txt" 2>&1
timeout -k 10 300 python3 bench.py "$@" > "$OUT/bench.json" 2> "$OUT/bench.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run \
  -- python3 bench.py --steps 10 --warmup 2 --no-cpu --no-extras "$@" > "$OUT/bench_under_rocprof.json" 2> "$OUT/rocprof_trace.err"
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "scale_kernel|wave_kernel" --output-format csv \
  -d "$OUT/pmc/fetch" -o pmc -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-extras "$@" > /dev/null 2> "$OUT/rocprof_fetch.err"
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "scale_kernel|wave_kernel" --output-format csv \
  -d "$OUT/pmc/write" -o pmc -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-extras "$@" > /dev/null 2> "$OUT/rocprof_write.err"
tools/iter_cost.sh "$OUT/iter" > "$OUT/iter_cost.txt" 2>&1
bash tools/pmc_lds.sh "$OUT/lds" > "$OUT/lds_cost.txt" 2>&1
echo done
