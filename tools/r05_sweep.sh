#!/bin/bash
# Scale kernel gradient sweep: state vector in every lane of wave 0 (product) vs the LDS lane rows
# (MPCQP_SCALE_LDS_SWEEP): phase timing of both, then bench A/B at N = 10 and 20.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/sweep
mkdir -p $O
MPCQP_LIB=$PWD/exp/sct10.so timeout -k 10 120 python3 tools/scale_phases.py $O/phases_lds.json > /dev/null 2>&1 || exit 1
MPCQP_LIB=$PWD/exp/swt10.so timeout -k 10 120 python3 tools/scale_phases.py $O/phases_reg.json > /dev/null 2>&1 || exit 1
python3 -c "
import json; a=json.load(open('$O/phases_lds.json')); b=json.load(open('$O/phases_reg.json'))
for k in a: print(k, a[k], b[k])"
AB_TAG=sw timeout -k 10 900 tools/r05_ab.sh 10 3 sw10 ub10 sw10w3 || exit 1
AB_TAG=sw timeout -k 10 700 tools/r05_ab.sh 20 2 sw20 ub20 || exit 1
