#!/bin/bash
# Two-phase solve A/B (MPCQP_PARK = the park iteration; 0 = one phase): GPU tests of the park path,
# one parity run per setting (oracle on 4096 robots), then interleaved timing runs of C2, C5 and the
# C3 shard.   usage: tools/r06_park_ab.sh OUTDIR REPS CUT...
set -euo pipefail
export TMPDIR=/tmp
O=${1:?outdir}; REPS=$2; shift 2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_park.py -v --timeout 200 --timeout-method thread > $O/park_tests.txt 2>&1 || { tail -30 $O/park_tests.txt; exit 1; }
grep -E "passed|failed" $O/park_tests.txt | tail -2
summ() {
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); p=d.get('parity') or {}; print(sys.argv[2], round(d['value']), 'ms', round(d['ms_per_step'], 4), 'err', p.get('max_rel_err_u0'), 'iters_equal', p.get('iters_equal'))" "$1" "$2"
}
for c in "$@"; do
  MPCQP_PARK=$c timeout -k 10 200 python3 bench.py --no-extras --cpu-sample 32 > $O/par_$c.json 2> $O/par_$c.err
  summ $O/par_$c.json "C2 park=$c parity"
done
for rep in $(seq 1 $REPS); do
  for c in "$@"; do
    MPCQP_PARK=$c timeout -k 10 120 python3 bench.py --no-cpu --no-extras > $O/c2_$c.$rep.json 2> /dev/null
    summ $O/c2_$c.$rep.json "C2 park=$c rep=$rep"
    MPCQP_PARK=$c timeout -k 10 120 python3 bench.py --no-cpu --no-extras --gait mixed --mixed-mu --batch 8192 > $O/c5_$c.$rep.json 2> /dev/null
    summ $O/c5_$c.$rep.json "C5 park=$c rep=$rep"
    MPCQP_PARK=$c timeout -k 10 120 python3 bench.py --no-cpu --no-extras --batch 8192 > $O/c3_$c.$rep.json 2> /dev/null
    summ $O/c3_$c.$rep.json "C3shard park=$c rep=$rep"
  done
done
