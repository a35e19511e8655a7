#!/bin/bash
# Setup without the scratch copy of the row-4 operands (new10) against the previous build (old10):
# GPU tests on the product library, bench A/B at N = 10, HBM traffic of both.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/scr
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
AB_TAG=scr timeout -k 10 900 tools/r05_ab.sh 10 4 new10 old10 || exit 1
for v in new10 old10; do
  MPCQP_LIB=$PWD/exp/$v.so timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "scale_kernel|wave_kernel" --output-format csv \
    -d $O/$v/pmc/write -o pmc -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-extras > /dev/null 2> $O/$v.write.err || exit 1
  MPCQP_LIB=$PWD/exp/$v.so timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "scale_kernel|wave_kernel" --output-format csv \
    -d $O/$v/pmc/fetch -o pmc -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-extras > /dev/null 2> $O/$v.fetch.err || exit 1
done
