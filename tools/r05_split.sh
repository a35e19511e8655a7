#!/bin/bash
# Round-5 batch-split experiments (tools/split_exp.py) over the bench configurations, after the
# split tests.  Output under gpurun_out/split/.
set -o pipefail
mkdir -p gpurun_out/split
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_split.py > gpurun_out/split/test.txt 2>&1 && \
timeout -k 10 200 python3 tools/split_exp.py --batch 4096 --ks 1 2 3 4 1 3 4 > gpurun_out/split/c2.txt 2>&1 && \
timeout -k 10 200 python3 tools/split_exp.py --batch 8192 --ks 1 2 3 4 > gpurun_out/split/c3.txt 2>&1 && \
timeout -k 10 200 python3 tools/split_exp.py --batch 8192 --gait mixed --mixed-mu --seed 4000 --ks 1 2 3 4 > gpurun_out/split/c5.txt 2>&1 && \
timeout -k 10 300 python3 tools/split_exp.py --batch 4096 --horizon 20 --ks 1 2 3 4 --steps 10 > gpurun_out/split/c4.txt 2>&1 && \
timeout -k 10 300 python3 tools/split_exp.py --batch 65536 --ks 1 3 4 --steps 5 > gpurun_out/split/big.txt 2>&1
rc=$?
tail -3 gpurun_out/split/test.txt; cat gpurun_out/split/c*.txt gpurun_out/split/big.txt 2>/dev/null | grep -v amdgpu.ids
exit $rc
