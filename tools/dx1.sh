set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/dx1
timeout -k 10 300 python -u -m pytest tests/test_gpu_dx.py -x -v --timeout 120 --timeout-method thread > gpurun_out/dx1/tests.txt 2>&1
rc=$?
tail -5 gpurun_out/dx1/tests.txt
timeout -k 10 200 python bench.py --solver dx --steps 10 --warmup 2 --no-cpu > gpurun_out/dx1/bench_dx.json 2> gpurun_out/dx1/bench_dx.err
echo "bench rc $?"
timeout -k 10 200 python bench.py --solver wave --steps 10 --warmup 2 --no-cpu > gpurun_out/dx1/bench_wave.json 2> gpurun_out/dx1/bench_wave.err
echo "bench rc $?"
exit $rc
