#!/bin/bash
# hand-off threshold vs C5 rate and accuracy (stance / mixed, state weights x1, x5, x100)
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/thr
mkdir -p $O
for L in go1-qp-mpc-controller_amd/lib/libmpcqp.so variants/g_3e4.so variants/g_1e5.so variants/g_3e5.so variants/nocheck.so; do
  b=$(basename $L .so)
  MPCQP_LIB=$L timeout -k 10 300 python3 -u tools/fuzz_parity.py --seeds 4 --batch 512 --horizons 10 --gaits stance,mixed --scales 1,5,100 > $O/fuzz_$b.log 2>&1
  MPCQP_LIB=$L timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu --no-extras --gait mixed --mixed-mu --batch 8192 > $O/c5_$b.json 2> $O/c5_$b.err
done
echo done
