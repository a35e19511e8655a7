#!/bin/bash
# Phase timing (timing builds exp/r5_pt10.so, exp/r5_pt20.so) and the VALU microbenchmark.
set -euo pipefail
export TMPDIR=/tmp
OUT=${1:?outdir}
mkdir -p "$OUT"
timeout -k 10 60 tools/mb/mb_valu > "$OUT/mb_valu.txt" 2>&1 && cat "$OUT/mb_valu.txt"
MPCQP_LIB=$PWD/exp/r5_pt10.so timeout -k 10 120 python3 tools/wave_phases.py --out "$OUT/phases_n10.json" > "$OUT/phases_n10.txt" 2>&1
MPCQP_LIB=$PWD/exp/r5_pt20.so timeout -k 10 120 python3 tools/wave_phases.py --horizon 20 --out "$OUT/phases_n20.json" > "$OUT/phases_n20.txt" 2>&1
python3 -c "
import json
for n in ('n10','n20'):
    d=json.load(open('$OUT/phases_'+n+'.json')); print(n, {k: round(v) for k,v in d.items() if k not in ('shader_ghz',)})"
