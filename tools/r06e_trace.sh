set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r06e; mkdir -p $O
for c in 0 50; do
MPCQP_PARK=$c timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t$c -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-extras > $O/b$c.json 2> $O/e$c.err
done
python3 - << 'PY'
import csv,glob
for c in (0,50):
    f=glob.glob(f"gpurun_out/r06e/t{c}/**/run_kernel_trace.csv",recursive=True)[0]
    rows=list(csv.DictReader(open(f)))
    rows=[r for r in rows if 'kernel' in r['Kernel_Name']]
    rows.sort(key=lambda r:int(r['Start_Timestamp']))
    t0=int(rows[0]['Start_Timestamp'])
    for r in rows[-8:]:
        print(c, r['Kernel_Name'][:40], (int(r['Start_Timestamp'])-t0)/1e3, (int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3)
PY
