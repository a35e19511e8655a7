#!/bin/bash
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r06k; mkdir -p $O
MPCQP_SENTINEL_LOG=$PWD/$O/sent_contract_on.jsonl MPCQP_LIB=$PWD/exp/contract_on.so timeout -k 10 300 \
  python -u -m pytest tests/test_gpu_conditioning.py tests/test_gpu_parity.py tests/test_gpu_degenerate.py tests/test_gpu_golden_fullsize.py -q --timeout 200 --timeout-method thread > $O/tests_contract_on.txt 2>&1 || true
tail -3 $O/tests_contract_on.txt
bash tools/r06_run.sh gpurun_out/r06k/main r05
