#!/bin/bash
# Time-sliced Schur wave kernel (round robin over the batch): bitwise A/B against the previous
# build, kernel time vs slice length (MPCQP_SLICE; 0 = one robot per workgroup, no slicing), batch
# scaling, GPU tests
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/slice
mkdir -p $O
L=go1-qp-mpc-controller_amd/lib/libmpcqp.so
MPCQP_LIB=variants/pre_fixed.so timeout -k 10 200 python3 tools/ab_bitwise.py dump $O/old.npz > $O/dump_old.txt 2>&1
timeout -k 10 200 python3 tools/ab_bitwise.py dump $O/new.npz > $O/dump_new.txt 2>&1
python3 tools/ab_bitwise.py cmp $O/old.npz $O/new.npz > $O/cmp.txt 2>&1 || true
for S in 0 50 75 100; do
  MPCQP_SLICE=$S timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu --no-extras > $O/b_s$S.json 2> $O/b_s$S.err
done
MPCQP_LIB=variants/pre_fixed.so timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu --no-extras > $O/b_pre.json 2> $O/b_pre.err
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1
echo done
