#!/bin/bash
# scale_kernel occupancy variants (HREG off, waves per SIMD) at N = 10 / 20, then the GPU tests of
# the product library (Acl-free Riccati form at N = 20 by default)
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/occ
mkdir -p $O
L=go1-qp-mpc-controller_amd/lib/libmpcqp.so
bash tools/ab_scale_tpc.sh $O/k10 10 $L variants/s10_h0_t2_w4.so variants/s10_h0_t1_w4.so variants/s10_h0_t1_w2.so > $O/k10.txt 2>&1
bash tools/ab_scale_tpc.sh $O/k20 20 $L variants/s20_t1_w4.so variants/s20_t1_w3.so > $O/k20.txt 2>&1
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1
echo done
