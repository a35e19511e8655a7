#!/bin/bash
# MFMA Gauss-Jordan A/B.  For each variant V (exp/V.so): C2 / C5 parity against
# the oracle and the GPU suite; phase timing of exp/gj0_t.so and exp/V_t.so; interleaved C2 / C5
# timing of the product library and the variants; the MFMA instruction count of the first variant.
#   usage: tools/r06_gj_ab.sh OUTDIR REPS V...
set -euo pipefail
export TMPDIR=/tmp
O=${1:?outdir}; REPS=$2; shift 2
mkdir -p $O
summ() {
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); p=d.get('parity') or {}; print(sys.argv[2], round(d['value']), 'ms', round(d['ms_per_step'], 4), 'err', p.get('max_rel_err_u0'), 'iters_equal', p.get('iters_equal'), p.get('iters_equal_frac'), 'handoff', (d.get('stats') or {}).get('handoff_count'))" "$1" "$2"
}
lib() { if [ "$1" = prod ]; then echo $PWD/go1-qp-mpc-controller_amd/lib/libmpcqp.so; else echo $PWD/exp/$1.so; fi; }
for v in "$@"; do
  MPCQP_LIB=$(lib $v) timeout -k 10 200 python3 bench.py --no-extras > $O/c2par_$v.json 2> $O/c2par_$v.err
  summ $O/c2par_$v.json "$v C2 parity"
  MPCQP_LIB=$(lib $v) timeout -k 10 200 python3 bench.py --no-extras --gait mixed --mixed-mu --batch 8192 > $O/c5par_$v.json 2> /dev/null
  summ $O/c5par_$v.json "$v C5 parity"
  MPCQP_SENTINEL_LOG=$PWD/$O/sent_$v.jsonl MPCQP_LIB=$(lib $v) timeout -k 10 400 \
    python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/tests_$v.txt 2>&1 || true
  echo "$v tests: $(grep -E "passed|failed" $O/tests_$v.txt | tail -1)"
  grep -E "^FAILED" $O/tests_$v.txt | head -10 || true
done
for v in gj0 "$@"; do
  MPCQP_LIB=$(lib ${v}_t) timeout -k 10 200 python3 tools/wave_phases.py --out $O/phases_$v.json > /dev/null 2> $O/phases_$v.err
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], {k: round(d[k]) for k in ('total','factor','f_pre','f_buildS','f_gj','f_post','iter_cycles') if k in d}, 'fact/robot', round(d['factorizations_per_robot'], 2))" $O/phases_$v.json ${v}_t
done
for rep in $(seq 1 $REPS); do
  for v in prod "$@"; do
    MPCQP_LIB=$(lib $v) timeout -k 10 120 python3 bench.py --no-cpu --no-extras > $O/c2_$v.$rep.json 2> /dev/null
    summ $O/c2_$v.$rep.json "$v C2 rep=$rep"
    MPCQP_LIB=$(lib $v) timeout -k 10 120 python3 bench.py --no-cpu --no-extras --gait mixed --mixed-mu --batch 8192 > $O/c5_$v.$rep.json 2> /dev/null
    summ $O/c5_$v.$rep.json "$v C5 rep=$rep"
  done
done
MPCQP_LIB=$(lib $1) timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU SQ_WAVE_CYCLES \
  --kernel-include-regex "wave_kernel" --output-format csv -d "$O/pmc" -o pmc -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-extras \
  > /dev/null 2> "$O/pmc.err"
python3 - "$O/pmc" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)
tot = collections.defaultdict(float); n = collections.Counter()
for row in csv.DictReader(open(f[0])):
    k = (row["Kernel_Name"][:60], row["Counter_Name"]); tot[k] += float(row["Counter_Value"]); n[k] += 1
for k in sorted(tot): print(k, "per dispatch %.4g" % (tot[k] / n[k]))
PY
