#!/bin/bash
# Round-5 batch-split ordering: concurrent parts vs chained parts (part i's scale_kernel after part
# i-1's, beside part i-1's wave_kernel), tools/split_exp.py at C2, C5 and C4.
set -o pipefail
mkdir -p gpurun_out/chain
for c in 0 1 0 1; do
  MPCQP_SPLIT_CHAIN=$c timeout -k 10 200 python3 tools/split_exp.py --batch 4096 --ks 1 2 3 > gpurun_out/chain/c2_$c.txt 2>&1 || exit $?
  echo "chain=$c"; grep -v amdgpu gpurun_out/chain/c2_$c.txt
done
for c in 0 1; do
  MPCQP_SPLIT_CHAIN=$c timeout -k 10 200 python3 tools/split_exp.py --batch 8192 --gait mixed --mixed-mu --seed 4000 --ks 1 3 > gpurun_out/chain/c5_$c.txt 2>&1 || exit $?
  echo "chain=$c"; grep -v amdgpu gpurun_out/chain/c5_$c.txt
  MPCQP_SPLIT_CHAIN=$c timeout -k 10 300 python3 tools/split_exp.py --batch 4096 --horizon 20 --ks 1 3 --steps 10 > gpurun_out/chain/c4_$c.txt 2>&1 || exit $?
  grep -v amdgpu gpurun_out/chain/c4_$c.txt
done
