#!/bin/bash
# P~dx fused into the check's P~x pass (schur_px2, product) vs computed apart (MPCQP_PDX_APART):
# GPU tests with sentinels on the product library, bench A/B at C2 and at C5's shape.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pdx
mkdir -p $O
export MPCQP_SENTINEL_LOG="$PWD/$O/sentinels.jsonl"
rm -f "$MPCQP_SENTINEL_LOG"
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
unset MPCQP_SENTINEL_LOG
AB_TAG=pdx timeout -k 10 900 tools/r05_ab.sh 10 4 fused10 apart10 || exit 1
BENCH_ARGS="--batch 8192 --gait mixed --mixed-mu" AB_TAG=pdx5 timeout -k 10 900 tools/r05_ab.sh 10 2 fused10 apart10 || exit 1
