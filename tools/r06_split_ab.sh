set -euo pipefail
export TMPDIR=/tmp
summ() {
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], round(d['value']), 'ms', round(d['ms_per_step'], 4))" "$1" "$2"
}
mkdir -p gpurun_out/r06n
for rep in 1 2; do
for sp in 3 4 5 2; do
  MPCQP_SPLIT=$sp timeout -k 10 120 python3 bench.py --no-cpu --no-extras > gpurun_out/r06n/c2_$sp.$rep.json 2>/dev/null
  summ gpurun_out/r06n/c2_$sp.$rep.json "C2 split=$sp rep=$rep"
  MPCQP_SPLIT=$sp timeout -k 10 120 python3 bench.py --no-cpu --no-extras --gait mixed --mixed-mu --batch 8192 > gpurun_out/r06n/c5_$sp.$rep.json 2>/dev/null
  summ gpurun_out/r06n/c5_$sp.$rep.json "C5 split=$sp rep=$rep"
done
done
