#!/bin/bash
# Round-5 hand-off threshold (MPCQP_SCHUR_SMAX) sweep: accuracy on the golden fixtures and the C2 /
# C5 rates of exp/ variants.
set -o pipefail
mkdir -p gpurun_out/acc
bash tools/r05_acc.sh "$@" > gpurun_out/acc/smax_acc.txt 2>&1; rc=$?
grep -E "^r5_|go1_mixed.npz|8192 mixed" gpurun_out/acc/smax_acc.txt
[ $rc -eq 0 ] || exit $rc
AB_TAG=_c5 BENCH_ARGS="--batch 8192 --gait mixed --mixed-mu" bash tools/r05_ab.sh 10 2 "$@"
