#!/bin/bash
# cost of the Schur conditioning handoff check: interleaved bench runs, no check vs check
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/abchk
mkdir -p $O
for rep in 1 2 3; do
  for L in variants/nocheck.so variants/check_v7.so; do
    b=$(basename $L .so)
    MPCQP_LIB=$L timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu --no-extras > $O/${b}_$rep.json 2> $O/${b}_$rep.err
  done
done
echo done
MPCQP_LIB=variants/check_v7.so timeout -k 10 400 python3 -u tools/fuzz_parity.py --seeds 6 --batch 512 --horizons 10 --gaits stance,mixed,trot --scales 100,1 > $O/fuzz_v7.log 2>&1
