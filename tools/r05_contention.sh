#!/bin/bash
# Per-robot phase costs of wave_kernel<10, 1> with 4 robots per CU (the product occupancy) against
# 2 and 1 robots per CU (dynamic-LDS padding, MPCQP_WAVE_LDS_PAD): what neighbours sharing a CU's
# LDS and instruction cache cost each robot.  Timing builds in exp/ (tools/build_variant.sh).
#   usage: tools/r05_contention.sh OUTDIR
set -euo pipefail
export TMPDIR=/tmp
OUT=${1:?outdir}
mkdir -p "$OUT"
for v in r5_pt r5_pt_pad2 r5_pt_pad1 r5_ends r5_ends_pad1; do
  MPCQP_LIB=$PWD/exp/$v.so timeout -k 10 120 python3 tools/wave_phases.py --out "$OUT/$v.json" > "$OUT/$v.txt" 2>&1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], {k: round(d[k]) for k in ('total','factor','f_gj','iter_cycles','check75','it_kkt','it_update','it_rest') if k in d})" "$OUT/$v.json" "$v"
done
