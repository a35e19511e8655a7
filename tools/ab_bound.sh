#!/bin/bash
# Round-4 A/B pass: per-foot bound-decided Ruiz passes (bitwise vs the previous library, kernel
# stats at N = 10 / 20, scale phases at N = 10), N = 20 phase timing, the Acl-free Riccati variant
# at N = 20, then the GPU tests
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/bound
mkdir -p $O gpurun_out/n20prof
MPCQP_LIB=variants/pre_bound.so timeout -k 10 200 python3 tools/ab_bitwise.py dump $O/old.npz > $O/dump_old.txt 2>&1
timeout -k 10 200 python3 tools/ab_bitwise.py dump $O/new.npz > $O/dump_new.txt 2>&1
python3 tools/ab_bitwise.py cmp $O/old.npz $O/new.npz > $O/cmp.txt 2>&1 || true
bash tools/ab_scale_tpc.sh $O/k10 10 variants/pre_bound.so go1-qp-mpc-controller_amd/lib/libmpcqp.so > $O/k10.txt 2>&1
MPCQP_LIB=variants/n10_sct.so timeout -k 10 200 python3 tools/scale_phases.py $O/scale_phases_n10.json > $O/scale_phases_n10.txt 2>&1
bash tools/ab_scale_tpc.sh $O/k20 20 variants/pre_bound.so variants/n20_cur.so variants/n20_noacl.so > $O/k20.txt 2>&1
MPCQP_LIB=variants/n20_pt.so timeout -k 10 200 python3 tools/wave_phases.py --horizon 20 --out gpurun_out/n20prof/wave_phases.json > gpurun_out/n20prof/wave_phases.txt 2>&1
MPCQP_LIB=variants/n20_noacl_pt.so timeout -k 10 200 python3 tools/wave_phases.py --horizon 20 --out gpurun_out/n20prof/wave_phases_noacl.json > gpurun_out/n20prof/wave_phases_noacl.txt 2>&1
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1
echo done
