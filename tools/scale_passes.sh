set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/scp
for sc in 0 1 10; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/scp/s$sc -o run -- python3 tools/scale_passes.py $sc > /dev/null 2>&1 || exit 1
  echo "scaling=$sc $(grep scale_kernel gpurun_out/scp/s$sc/run_kernel_stats.csv | cut -d, -f4)"
done
