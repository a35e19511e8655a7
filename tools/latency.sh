# kernel time vs batch for the wave (one wave per robot) and mw (one wave per round) solvers
set -uo pipefail
O=gpurun_out/lat; mkdir -p $O
for s in wave mw; do
  for b in 256 1024 2048 4096 8192; do
    timeout -k 10 120 python bench.py --solver $s --batch $b --no-cpu --steps 10 > $O/$s.$b.json 2> $O/$s.$b.err || exit 1
    python -c "import json; d=json.load(open('$O/$s.$b.json')); print('$s', $b, round(d['ms_per_step'],3), round(d['value']))"
  done
done
