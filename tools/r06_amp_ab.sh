#!/bin/bash
# Hand-off bound A/B (exp/NAME.so, horizon-10 builds): conditioning / golden sentinels per variant,
# C5 parity, then interleaved C2 and C5 timing.   usage: tools/r06_amp_ab.sh OUTDIR REPS NAME...
set -euo pipefail
export TMPDIR=/tmp
O=${1:?outdir}; REPS=$2; shift 2
mkdir -p $O
summ() {
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); p=d.get('parity') or {}; print(sys.argv[2], round(d['value']), 'ms', round(d['ms_per_step'], 4), 'err', p.get('max_rel_err_u0'), 'iters_equal', p.get('iters_equal'), 'handoff', (d.get('stats') or {}).get('handoff_count'))" "$1" "$2"
}
for v in "$@"; do
  MPCQP_SENTINEL_LOG=$PWD/$O/sent_$v.jsonl MPCQP_SENTINEL_CALIBRATE=1 MPCQP_LIB=$PWD/exp/$v.so timeout -k 10 300 \
    python -u -m pytest tests/test_gpu_conditioning.py tests/test_gpu_parity.py -q --timeout 200 --timeout-method thread > $O/tests_$v.txt 2>&1 || true
  python3 -c "
import json,sys
rows=[json.loads(l) for l in open(sys.argv[1])]
w=max((r for r in rows if 'max_rel_err_u0' in r and 'warm' not in r['label']), key=lambda r: r['max_rel_err_u0'])
print(sys.argv[2], 'worst cold sentinel', w['label'], '%.2e' % w['max_rel_err_u0'], '| tests:', open(sys.argv[3]).read().strip().splitlines()[-1])" $O/sent_$v.jsonl $v $O/tests_$v.txt
  MPCQP_LIB=$PWD/exp/$v.so timeout -k 10 200 python3 bench.py --no-extras --cpu-sample 32 --gait mixed --mixed-mu --batch 8192 > $O/c5par_$v.json 2> /dev/null
  summ $O/c5par_$v.json "$v C5 parity"
done
for rep in $(seq 1 $REPS); do
  for v in "$@"; do
    MPCQP_LIB=$PWD/exp/$v.so timeout -k 10 120 python3 bench.py --no-cpu --no-extras > $O/c2_$v.$rep.json 2> /dev/null
    summ $O/c2_$v.$rep.json "$v C2 rep=$rep"
    MPCQP_LIB=$PWD/exp/$v.so timeout -k 10 120 python3 bench.py --no-cpu --no-extras --gait mixed --mixed-mu --batch 8192 > $O/c5_$v.$rep.json 2> /dev/null
    summ $O/c5_$v.$rep.json "$v C5 rep=$rep"
  done
done
