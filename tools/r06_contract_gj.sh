#!/bin/bash
# -ffp-contract=on build of the final product source (exp/contract_on.so, `make variant
# DEFS=-ffp-contract=on`): the accuracy / hand-off GPU tests with their sentinels.
#   usage: tools/r06_contract_gj.sh OUTDIR
set -euo pipefail
export TMPDIR=/tmp
O=${1:?outdir}; mkdir -p $O
MPCQP_SENTINEL_LOG=$PWD/$O/sent_contract_on.jsonl MPCQP_LIB=$PWD/exp/contract_on.so timeout -k 10 300 \
  python -u -m pytest tests/test_gpu_conditioning.py tests/test_gpu_parity.py tests/test_gpu_degenerate.py tests/test_gpu_golden_fullsize.py -q --timeout 200 --timeout-method thread > $O/tests_contract_on.txt 2>&1 || true
tail -1 $O/tests_contract_on.txt
