#!/bin/bash
# Round-5 accuracy check of exp/ variants: the golden-fixture tests with the sentinels in
# calibration mode (errors printed, not asserted), then the N = 10 A/B.
#   usage: tools/r05_acc.sh NAME...
set -o pipefail
mkdir -p gpurun_out/acc
for v in "$@"; do
  MPCQP_LIB=$PWD/exp/$v.so MPCQP_SENTINEL_CALIBRATE=1 MPCQP_SENTINEL_LOG=$PWD/gpurun_out/acc/$v.jsonl \
    timeout -k 10 300 python3 -u -m pytest -q -s --timeout 120 --timeout-method thread tests/test_gpu_golden_fullsize.py tests/test_gpu_parity.py \
    -k "not n20 and not c4 and not other_horizons" > gpurun_out/acc/$v.txt 2>&1
  rc=$?; [ $rc -le 1 ] || exit $rc
  echo "$v"; grep -h "sentinel" gpurun_out/acc/$v.txt | head -12
done
bash tools/r05_ab.sh 10 2 "$@"
