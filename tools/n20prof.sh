set -euo pipefail
mkdir -p gpurun_out/n20prof
MPCQP_LIB=variants/n20_pt.so timeout -k 10 200 python3 tools/wave_phases.py --horizon 20 --out gpurun_out/n20prof/wave_phases.json > gpurun_out/n20prof/wave_phases.txt 2>&1
MPCQP_N=20 MPCQP_LIB=variants/n20_sct.so timeout -k 10 200 python3 tools/scale_phases.py gpurun_out/n20prof/scale_phases.json > gpurun_out/n20prof/scale_phases.txt 2>&1
echo ok
