#!/bin/bash
# Ruiz passes stopped at an exact fixed point: bitwise A/B vs the previous build, kernel stats,
# scale phases at N = 10, GPU tests
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/fixed
mkdir -p $O
L=go1-qp-mpc-controller_amd/lib/libmpcqp.so
MPCQP_LIB=variants/pre_fixed.so timeout -k 10 200 python3 tools/ab_bitwise.py dump $O/old.npz > $O/dump_old.txt 2>&1
timeout -k 10 200 python3 tools/ab_bitwise.py dump $O/new.npz > $O/dump_new.txt 2>&1
python3 tools/ab_bitwise.py cmp $O/old.npz $O/new.npz > $O/cmp.txt 2>&1 || true
bash tools/ab_scale_tpc.sh $O/k10 10 variants/pre_fixed.so $L > $O/k10.txt 2>&1
bash tools/ab_scale_tpc.sh $O/k20 20 variants/pre_fixed.so $L > $O/k20.txt 2>&1
MPCQP_LIB=variants/n10_sct.so timeout -k 10 200 python3 tools/scale_phases.py $O/scale_n10.json > $O/scale_n10.txt 2>&1
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1
echo done
