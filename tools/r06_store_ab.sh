#!/bin/bash
# Branch-free Q stores of the matrix-core Gauss-Jordan: GPU suite, then interleaved C2 / C5 timing of
# the product library against exp/gjs.so (masked stores).   usage: tools/r06_store_ab.sh OUT REPS
set -euo pipefail
export TMPDIR=/tmp
O=${1:?outdir}; REPS=$2
mkdir -p $O
summ() {
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); p=d.get('parity') or {}; print(sys.argv[2], round(d['value']), 'ms', round(d['ms_per_step'], 4), 'err', p.get('max_rel_err_u0'), 'iters_equal', p.get('iters_equal_frac'))" "$1" "$2"
}
lib() { if [ "$1" = prod ]; then echo $PWD/go1-qp-mpc-controller_amd/lib/libmpcqp.so; else echo $PWD/exp/$1.so; fi; }
timeout -k 10 120 tools/mb/mb_gjsweep > $O/mb_gjsweep.txt 2>&1
grep -E "median" $O/mb_gjsweep.txt
MPCQP_SENTINEL_LOG=$PWD/$O/sentinels.jsonl timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/gpu_tests.txt 2>&1
tail -1 $O/gpu_tests.txt
timeout -k 10 200 python3 bench.py --no-extras > $O/c2par.json 2> /dev/null
summ $O/c2par.json "prod C2 parity"
for rep in $(seq 1 $REPS); do
  for v in gjs prod; do
    MPCQP_LIB=$(lib $v) timeout -k 10 120 python3 bench.py --no-cpu --no-extras > $O/c2_$v.$rep.json 2> /dev/null
    summ $O/c2_$v.$rep.json "$v C2 rep=$rep"
    MPCQP_LIB=$(lib $v) timeout -k 10 120 python3 bench.py --no-cpu --no-extras --gait mixed --mixed-mu --batch 8192 > $O/c5_$v.$rep.json 2> /dev/null
    summ $O/c5_$v.$rep.json "$v C5 rep=$rep"
  done
done
