#!/bin/bash
# Round-4 evidence pass (through gpurun from the repo root): tools/profile_round.sh for C2, then the
# kernel-trace stats and FETCH_SIZE / WRITE_SIZE passes of the horizon-20 solve (C4).
#   usage: tools/profile_r04.sh OUTDIR
set -euo pipefail
export TMPDIR=/tmp
OUT=${1:?outdir}
bash tools/profile_round.sh "$OUT"
mkdir -p "$OUT/n20"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/n20/trace" -o run \
  -- python3 bench.py --steps 6 --warmup 2 --no-cpu --no-extras --horizon 20 > "$OUT/n20/bench_under_rocprof.json" 2> "$OUT/n20/rocprof_trace.err"
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "scale_kernel|wave_kernel" --output-format csv \
  -d "$OUT/n20/pmc/fetch" -o pmc -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-extras --horizon 20 > /dev/null 2> "$OUT/n20/rocprof_fetch.err"
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "scale_kernel|wave_kernel" --output-format csv \
  -d "$OUT/n20/pmc/write" -o pmc -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-extras --horizon 20 > /dev/null 2> "$OUT/n20/rocprof_write.err"
echo done
