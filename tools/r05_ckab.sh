#!/bin/bash
# Round-5 check-block experiments: A/B of exp/ variants at N = 10 plus phase timing of two timing
# builds (tools/wave_phases.py).
#   usage: tools/r05_ckab.sh REPS PT_A PT_B NAME...
set -euo pipefail
export TMPDIR=/tmp
REPS=$1; PA=$2; PB=$3; shift 3
mkdir -p gpurun_out/ckab
for v in $PA $PB; do
  MPCQP_LIB=$PWD/exp/$v.so timeout -k 10 120 python3 tools/wave_phases.py --out gpurun_out/ckab/$v.json > gpurun_out/ckab/$v.txt 2>&1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], {k: round(d[k]) for k in ('total','factor','f_gj','iter_cycles','check75','ck_px','ck_norms','ck_tests','ck_tail','it_kkt','it_update') if k in d})" gpurun_out/ckab/$v.json $v
done
bash tools/r05_ab.sh 10 $REPS "$@"
