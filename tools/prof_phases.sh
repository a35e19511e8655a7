#!/bin/bash
# scale_kernel phase timing at N = 10 / 20 and wave_kernel phase timing at N = 20 (timing builds)
set -euo pipefail
O=gpurun_out/phases
mkdir -p $O
MPCQP_LIB=variants/n10_sct.so timeout -k 10 200 python3 tools/scale_phases.py $O/scale_n10.json > $O/scale_n10.txt 2>&1
MPCQP_N=20 MPCQP_LIB=variants/n20_sct.so timeout -k 10 200 python3 tools/scale_phases.py $O/scale_n20.json > $O/scale_n20.txt 2>&1
MPCQP_LIB=variants/n20_pt.so timeout -k 10 200 python3 tools/wave_phases.py --horizon 20 --out $O/wave_n20.json > $O/wave_n20.txt 2>&1
echo done
