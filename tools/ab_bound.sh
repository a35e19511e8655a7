#!/bin/bash
# Bound-decided Ruiz passes: bitwise A/B against the previous library, kernel stats at N = 10 / 20
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/bound
mkdir -p $O
MPCQP_LIB=variants/pre_bound.so timeout -k 10 200 python3 tools/ab_bitwise.py dump $O/old.npz > $O/dump_old.txt 2>&1
timeout -k 10 200 python3 tools/ab_bitwise.py dump $O/new.npz > $O/dump_new.txt 2>&1
python3 tools/ab_bitwise.py cmp $O/old.npz $O/new.npz > $O/cmp.txt 2>&1 || true
bash tools/ab_scale_tpc.sh $O/k10 10 variants/pre_bound.so go1-qp-mpc-controller_amd/lib/libmpcqp.so > $O/k10.txt 2>&1
bash tools/ab_scale_tpc.sh $O/k20 20 variants/pre_bound.so go1-qp-mpc-controller_amd/lib/libmpcqp.so > $O/k20.txt 2>&1
bash tools/n20prof.sh
echo done
