#!/bin/bash
# Round-5 A/B of kernel variants (exp/NAME.so, single-horizon builds): one parity run per variant
# (oracle on 4096 robots), then REPS interleaved timing runs.
#   usage: tools/r05_ab.sh HORIZON REPS NAME...
set -euo pipefail
export TMPDIR=/tmp
H=$1; REPS=$2; shift 2
O=gpurun_out/ab$H${AB_TAG:-}
mkdir -p $O
summ() {
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); p=d.get('parity') or {}; print(sys.argv[2], round(d['value']), 'kernel_ms', round(d['roofline']['kernel_ms'], 4), 'iters', round(d['stats']['mean_iters'], 3), 'err', p.get('max_rel_err_u0'), 'iters_equal', p.get('iters_equal'))" "$1" "$2"
}
lib_of() { [ "$1" = product ] && echo "$PWD/go1-qp-mpc-controller_amd/lib/libmpcqp.so" || echo "$PWD/exp/$1.so"; }
for v in "$@"; do
  MPCQP_LIB=$(lib_of $v) timeout -k 10 200 python3 bench.py --horizon $H ${BENCH_ARGS:-} --no-extras --cpu-sample 32 > $O/$v.par.json 2> $O/$v.par.err
  summ $O/$v.par.json "$v parity"
done
for rep in $(seq 1 $REPS); do
  for v in "$@"; do
    MPCQP_LIB=$(lib_of $v) timeout -k 10 120 python3 bench.py --horizon $H ${BENCH_ARGS:-} --no-cpu --no-extras > $O/$v.$rep.json 2> $O/$v.$rep.err
    summ $O/$v.$rep.json "$v $rep"
  done
done
