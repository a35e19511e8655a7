set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for v in tpc2 tpc4; do
  MPCQP_LIB=$PWD/variants/$v.so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab/$v -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/ab/$v.json 2> gpurun_out/ab/$v.err
done
