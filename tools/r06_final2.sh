#!/bin/bash
# Round-6 final evidence after the MFMA Gauss-Jordan became the default: GPU suite with sentinels,
# smoke(), then tools/r06_final.sh.   usage: tools/r06_final2.sh OUTDIR
set -euo pipefail
export TMPDIR=/tmp
OUT=${1:?outdir}
mkdir -p "$OUT"
MPCQP_SENTINEL_LOG=$PWD/$OUT/sentinels.jsonl timeout -k 10 500 \
  python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > "$OUT/gpu_tests.txt" 2>&1
tail -1 "$OUT/gpu_tests.txt"
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.txt" 2>&1
tail -1 "$OUT/smoke.txt"
tools/r06_final.sh "$OUT"
