# SQ counters of wave_kernel (one --pmc pass per call, each under its own time limit)
#   tools/pmc_sq.sh OUTDIR "COUNTERS..." [bench args]
set -euo pipefail
export TMPDIR=/tmp
O=$1
CTR=$2
shift 2
mkdir -p "$O"
[ -f "$O/counters.txt" ] || timeout -s KILL 60 rocprofv3 -L > "$O/counters.txt" 2>&1 || true
tag=${KRE:-wave}_$(echo "$CTR" | tr ' ' '_' | cut -c1-60)
timeout -s KILL 120 rocprofv3 --pmc $CTR --kernel-include-regex "${KRE:-wave_kernel}" --output-format csv -d "$O/$tag" -o pmc \
  -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-extras "$@" > "$O/$tag.out" 2> "$O/$tag.err"
