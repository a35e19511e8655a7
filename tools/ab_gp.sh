#!/bin/bash
# Packed G^-1 (four robots per CU at N = 20) vs the full-G^-1 Acl-free form, and the scale passes
# that skip 1/sqrt(1), against the previous builds; bitwise A/B at N = 10; GPU tests; bench line
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/gp
mkdir -p $O
L=go1-qp-mpc-controller_amd/lib/libmpcqp.so
bash tools/ab_scale_tpc.sh $O/k20 20 variants/n20_noacl.so variants/s20_t1_w3.so $L > $O/k20.txt 2>&1
bash tools/ab_scale_tpc.sh $O/k10 10 variants/s10_h0_t1_w2.so $L > $O/k10.txt 2>&1
MPCQP_LIB=variants/pre_bound.so timeout -k 10 200 python3 tools/ab_bitwise.py dump $O/old.npz > $O/dump_old.txt 2>&1
timeout -k 10 200 python3 tools/ab_bitwise.py dump $O/new.npz > $O/dump_new.txt 2>&1
python3 tools/ab_bitwise.py cmp $O/old.npz $O/new.npz > $O/cmp.txt 2>&1 || true
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err
echo done
