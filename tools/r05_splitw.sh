#!/bin/bash
# Relative part sizes of the three-part batch split (MPCQP_SPLIT_W, read at handle creation):
# tools/split_exp.py per setting, interleaved twice.  Output under gpurun_out/splitw/.
set -o pipefail
mkdir -p gpurun_out/splitw
out=gpurun_out/splitw/c2.txt
: > $out
for rep in 1 2; do
  for w in 1,1,1 1,2,2 2,3,3 3,2,2 2,1,1 1,1,2 2,2,1 1,3,3; do
    echo "w=$w rep=$rep" >> $out
    MPCQP_SPLIT_W=$w timeout -k 10 120 python3 tools/split_exp.py --batch 4096 --ks 3 1 3 --steps 20 >> $out 2>&1 || exit 1
  done
done
grep -v amdgpu.ids $out
