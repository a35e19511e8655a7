#!/bin/bash
# Schur -> Riccati handoff threshold on max_i S_ii: u0 accuracy (stance, q x 100 / x 1 / trot) and
# C2 rate per threshold (variants built with -DMPCQP_SCHUR_SMAX=T at N = 10)
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/smax
mkdir -p $O
for L in go1-qp-mpc-controller_amd/lib/libmpcqp.so variants/smax_1e3.so variants/smax_1e4.so variants/smax_1e5.so variants/smax_1e6.so; do
  b=$(basename $L .so)
  MPCQP_LIB=$L timeout -k 10 300 python3 -u tools/fuzz_parity.py --seeds 4 --batch 512 --horizons 10 --gaits stance,trot,mixed --scales 100,1 > $O/fuzz_$b.log 2>&1
  MPCQP_LIB=$L timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu --no-extras > $O/bench_$b.json 2> $O/bench_$b.err
done
echo done
