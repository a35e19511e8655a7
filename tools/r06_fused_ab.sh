#!/bin/bash
# Fused scale_data A/B: bitwise dumps (exp/unfused.so vs exp/fused.so), the GPU tests against the
# fused library (horizons 1, 5, 10, 20 only in these builds), interleaved C2 / C5 / C3-shard timing
# and the fused C2 HBM traffic.   usage: tools/r06_fused_ab.sh OUTDIR REPS
set -euo pipefail
export TMPDIR=/tmp
O=${1:?outdir}; REPS=$2
mkdir -p $O
for v in unfused fused; do
  MPCQP_LIB=$PWD/exp/$v.so timeout -k 10 200 python3 tools/ab_bitwise.py dump $O/ab_$v.npz > $O/ab_$v.txt 2>&1
done
python3 tools/ab_bitwise.py cmp $O/ab_unfused.npz $O/ab_fused.npz > $O/ab.txt || true
cat $O/ab.txt; rm -f $O/ab_*.npz
MPCQP_SENTINEL_LOG=$PWD/$O/sent_fused.jsonl MPCQP_LIB=$PWD/exp/fused.so timeout -k 10 400 \
  python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/tests_fused.txt 2>&1 || true
grep -E "passed|failed" $O/tests_fused.txt | tail -1
grep -E "^FAILED" $O/tests_fused.txt | head -30 || true
summ() {
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); p=d.get('parity') or {}; print(sys.argv[2], round(d['value']), 'ms', round(d['ms_per_step'], 4), 'err', p.get('max_rel_err_u0'), 'iters_equal', p.get('iters_equal'))" "$1" "$2"
}
for v in unfused fused; do
  MPCQP_LIB=$PWD/exp/$v.so timeout -k 10 200 python3 bench.py --no-extras --cpu-sample 32 > $O/par_$v.json 2> /dev/null
  summ $O/par_$v.json "$v C2 parity"
done
for rep in $(seq 1 $REPS); do
  for v in unfused fused; do
    MPCQP_LIB=$PWD/exp/$v.so timeout -k 10 120 python3 bench.py --no-cpu --no-extras > $O/c2_$v.$rep.json 2> /dev/null
    summ $O/c2_$v.$rep.json "$v C2 rep=$rep"
    MPCQP_LIB=$PWD/exp/$v.so timeout -k 10 120 python3 bench.py --no-cpu --no-extras --gait mixed --mixed-mu --batch 8192 > $O/c5_$v.$rep.json 2> /dev/null
    summ $O/c5_$v.$rep.json "$v C5 rep=$rep"
    MPCQP_LIB=$PWD/exp/$v.so timeout -k 10 120 python3 bench.py --no-cpu --no-extras --batch 8192 > $O/c3_$v.$rep.json 2> /dev/null
    summ $O/c3_$v.$rep.json "$v C3shard rep=$rep"
  done
done
MPCQP_LIB=$PWD/exp/fused.so timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "wave_kernel" --output-format csv \
  -d "$O/pmc/fetch" -o pmc -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-extras > /dev/null 2> "$O/fetch.err"
MPCQP_LIB=$PWD/exp/fused.so timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "wave_kernel" --output-format csv \
  -d "$O/pmc/write" -o pmc -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-extras > /dev/null 2> "$O/write.err"
python3 tools/pmc_traffic.py "$O/pmc" --key N10_B4096_trot_fused --kernel wave_kernel --parts 3 --out "$O/pmc_traffic.json" | grep hbm_bytes
