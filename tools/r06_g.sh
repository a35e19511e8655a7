#!/bin/bash
set -euo pipefail
export TMPDIR=/tmp
bash tools/r06_park_ab.sh gpurun_out/r06f 2 0 50 100
bash tools/r06e_trace.sh
mkdir -p gpurun_out/r06g
MPCQP_LIB=$PWD/exp/cond_fast.so timeout -k 10 300 python3 -u tools/r06_cancel.py gpurun_out/r06g/cancel_fast.json > gpurun_out/r06g/cancel_fast.txt 2>&1
MPCQP_LIB=$PWD/exp/cond_on.so timeout -k 10 300 python3 -u tools/r06_cancel.py gpurun_out/r06g/cancel_on.json > gpurun_out/r06g/cancel_on.txt 2>&1
tail -40 gpurun_out/r06g/cancel_fast.txt
