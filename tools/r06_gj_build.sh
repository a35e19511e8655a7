#!/bin/bash
# Round-6 MFMA Gauss-Jordan A/B libraries (exp/*.so, not shipped), MFMA results in VGPRs:
#   gjs      MPCQP_GJ_MFMA=1 (blocked sweep on the matrix cores), every horizon
#   gjs_t    the same with phase timing, horizon 10;  gj0_t: product source, phase timing
#   vf             product source + MFMA results in VGPRs (the flag alone), horizons 1, 5, 10, 20
#   usage: tools/r06_gj_build.sh NAME...
set -euo pipefail
cd "$(dirname "$0")/../go1-qp-mpc-controller_amd"
mkdir -p ../exp
SRC="csrc/mpcqp_wave.hip csrc/mpcqp_build.hip csrc/mpcqp_torque.hip csrc/mpcqp_balance.hip csrc/mpcqp_assemble.hip -x hip csrc/mpcqp_capi.cpp"
FL="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -fno-strict-aliasing -shared"
VF="-mllvm -amdgpu-mfma-vgpr-form"
T="-DMPCQP_PHASE_TIMING"
N10="-DMPCQP_WAVE_FOR_EACH_N(X)=X(10)"
b() { local out=$1; shift; /opt/rocm/bin/hipcc $FL "$@" $SRC -o ../exp/$out.so && echo built $out; }
for v in "$@"; do
  case $v in
    gjs) b gjs -DMPCQP_GJ_MFMA=1 $VF & ;;
    gjs_t) b gjs_t -DMPCQP_GJ_MFMA=1 $VF $T "$N10" & ;;
    gj0_t) b gj0_t $T "$N10" & ;;
    vf) b vf $VF "-DMPCQP_WAVE_FOR_EACH_N(X)=X(1) X(5) X(10) X(20)" & ;;
  esac
done
wait
