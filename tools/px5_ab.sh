set -e
mkdir -p gpurun_out/px5_ab
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu > gpurun_out/px5_ab/parity.log 2>&1
for i in 1 2; do
LBF_LIB=$PWD/bitflood_amd/lib/ab/liblbfhash_px5_before.so timeout -k 10 200 python -u bench.py --config c4 --no-cpu-baseline --no-e2e > gpurun_out/px5_ab/before_$i.json 2> gpurun_out/px5_ab/before_$i.err
timeout -k 10 200 python -u bench.py --config c4 --no-cpu-baseline --no-e2e > gpurun_out/px5_ab/after_$i.json 2> gpurun_out/px5_ab/after_$i.err
done
