#!/bin/bash
# Round-6 first GPU call: the degenerate-feet investigation (product, no screen, Riccati only), the
# round-start bench line, and the executed-FP64 counter passes (C2, C4, plus the mb_valu calibration).
#   usage: tools/r06_first.sh OUTDIR
set -euo pipefail
export TMPDIR=/tmp
OUT=${1:?outdir}
mkdir -p "$OUT/flops"
timeout -k 10 300 python3 -u tools/r06_degen_sweep.py "$OUT/sweep_product.json" > "$OUT/sweep_product.txt" 2>&1
MPCQP_LIB=$PWD/exp/gtol0.so timeout -k 10 200 python3 -u tools/r06_degen_sweep.py "$OUT/sweep_gtol0.json" --no-large > "$OUT/sweep_gtol0.txt" 2>&1
MPCQP_LIB=$PWD/exp/ric.so timeout -k 10 200 python3 -u tools/r06_degen_sweep.py "$OUT/sweep_ric.json" --no-large > "$OUT/sweep_ric.txt" 2>&1
timeout -k 10 300 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
PMC="SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAVE_CYCLES"
timeout -s KILL 60 rocprofv3 --pmc $PMC --kernel-include-regex "k_fma|k_max" --output-format csv -d "$OUT/flops/calib" -o pmc \
  -- tools/mb/mb_valu > "$OUT/flops/mb_valu.txt" 2> "$OUT/flops/calib.err"
for H in 10 20; do
  timeout -s KILL 120 rocprofv3 --pmc $PMC --kernel-include-regex "scale_kernel|wave_kernel" --output-format csv \
    -d "$OUT/flops/h$H" -o pmc -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-extras --horizon $H \
    > "$OUT/flops/bench_h$H.json" 2> "$OUT/flops/h$H.err"
done
python3 tools/pmc_flops.py "$OUT/flops/h10" --key N10_B4096_trot --parts 3 --calib "$OUT/flops/calib" --out "$OUT/pmc_flops.json"
python3 tools/pmc_flops.py "$OUT/flops/h20" --key N20_B4096_trot --parts 3 --out "$OUT/pmc_flops.json"
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('bench', round(d['value']), d['ms_per_step'], d['roofline']['frac'])" "$OUT/bench.json"
