set -e
export TMPDIR=/tmp
O=gpurun_out/r2o; mkdir -p $O
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS --kernel-include-regex scale_kernel --output-format csv -d $O/s1 -o pmc -- python3 bench.py --steps 2 --warmup 1 --no-cpu > /dev/null 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT --kernel-include-regex scale_kernel --output-format csv -d $O/s2 -o pmc -- python3 bench.py --steps 2 --warmup 1 --no-cpu > /dev/null 2>&1
