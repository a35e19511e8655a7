#!/bin/bash
# A/B kernel variants on one box: bench.py (no CPU baseline, no extras) per library, interleaved
# over REPS rounds.  Variants are variants/NAME.so (make -C go1-qp-mpc-controller_amd variant
# OUT=../variants/NAME.so DEFS=...); "product" is the in-tree lib/libmpcqp.so.
#   tools/ab_bench.sh REPS NAME... [-- bench args]
set -uo pipefail
export TMPDIR=/tmp
REPS=$1
shift
names=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do names+=("$1"); shift; done
[ "${1:-}" = "--" ] && shift
mkdir -p gpurun_out/ab
for rep in $(seq 1 "$REPS"); do
  for v in "${names[@]}"; do
    lib=$PWD/exp/$v.so; [ -f "$lib" ] || lib=$PWD/variants/$v.so
    [ "$v" = product ] && lib=$PWD/go1-qp-mpc-controller_amd/lib/libmpcqp.so
    MPCQP_LIB=$lib timeout -k 10 120 python3 bench.py --no-cpu --no-extras "$@" > gpurun_out/ab/$v.$rep.json 2> gpurun_out/ab/$v.$rep.err || exit $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], round(d['value']), 'kernel_ms', round(d['roofline']['kernel_ms'], 4), 'iters', d['stats']['mean_iters'], 'parity', d.get('parity', {}).get('max_rel_u0') if isinstance(d.get('parity'), dict) else d.get('parity'))" gpurun_out/ab/$v.$rep.json "$v" "$rep"
  done
done
