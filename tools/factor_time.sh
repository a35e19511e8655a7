# wave_kernel time at max_iter=1 (setup + one factorization + one iteration) and scale_kernel time
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ft
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ft/s -o run -- python3 tools/scale_passes.py 10 > /dev/null 2>&1 || exit 1
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/ft/s/run_kernel_stats.csv')):
    if 'wave_kernel' in r['Name'] or 'scale_kernel' in r['Name']: print(r['Name'][:34], r['AverageNs'])"
