#!/bin/bash
# scale_kernel<20> at two waves per SIMD (256 VGPRs, no spills, two robots per CU) against three
# (168 VGPRs, 43 spilled): bench A/B at N = 20 and the HBM traffic of both.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/w20
mkdir -p $O
AB_TAG=w20 timeout -k 10 900 tools/r05_ab.sh 20 3 w2_20 w3_20 || exit 1
for v in w2_20 w3_20; do
  MPCQP_LIB=$PWD/exp/$v.so timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "scale_kernel|wave_kernel" --output-format csv \
    -d $O/$v/pmc/write -o pmc -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-extras --horizon 20 > /dev/null 2> $O/$v.write.err || exit 1
  MPCQP_LIB=$PWD/exp/$v.so timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "scale_kernel|wave_kernel" --output-format csv \
    -d $O/$v/pmc/fetch -o pmc -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-extras --horizon 20 > /dev/null 2> $O/$v.fetch.err || exit 1
  MPCQP_LIB=$PWD/exp/$v.so timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v/trace -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-extras --horizon 20 > /dev/null 2> $O/$v.trace.err || exit 1
  grep -h -E "scale_kernel|wave_kernel" $O/$v/trace/run_kernel_stats.csv | cut -c1-160
done
