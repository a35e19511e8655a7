set -e
export TMPDIR=/tmp
O=gpurun_out/r2pmc
mkdir -p $O
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU --kernel-include-regex wave_kernel --output-format csv -d $O/a -o pmc -- python3 bench.py --steps 2 --warmup 1 --no-cpu > $O/a.out 2> $O/a.err
