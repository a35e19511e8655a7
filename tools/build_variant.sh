#!/bin/bash
# Experiment build of the product library at one horizon (not shipped):
#   tools/build_variant.sh OUT.so N [-DFOO ...]
set -euo pipefail
OUT=${1:?out}; N=${2:?horizon}; shift 2
cd "$(dirname "$0")/../go1-qp-mpc-controller_amd"
mkdir -p "$(dirname "$OUT")"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -fno-strict-aliasing \
  "-DMPCQP_WAVE_FOR_EACH_N(X)=X($N)" "$@" -shared csrc/mpcqp_wave.hip csrc/mpcqp_build.hip csrc/mpcqp_torque.hip \
  csrc/mpcqp_balance.hip csrc/mpcqp_assemble.hip -x hip csrc/mpcqp_capi.cpp -o "$OUT"
