#!/bin/bash
# Scale kernel: raw column norms bounded from H's diagonal (product) vs exact (MPCQP_SCALE_EXACT_CM0):
# GPU tests on the product library, bench A/B at N = 10 and 20, kernel stats of both N = 10 builds.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/cm0
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }
tail -3 $O/gpu_tests.txt
AB_TAG=cm0 timeout -k 10 700 tools/r05_ab.sh 10 3 ub10 ex10 || exit 1
AB_TAG=cm0 timeout -k 10 700 tools/r05_ab.sh 20 2 ub20 ex20 || exit 1
for v in ub10 ex10; do
  MPCQP_LIB=$PWD/exp/$v.so timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -o run -- python3 bench.py --no-cpu --no-extras --steps 10 > $O/prof_$v.log 2>&1 || exit 1
  grep -h -E "scale_kernel|wave_kernel" $(find $O/prof_$v -name "*kernel_stats.csv") | cut -c1-200
done
