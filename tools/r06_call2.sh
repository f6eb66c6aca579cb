set -o pipefail
mkdir -p gpurun_out/r06c2
export TMPDIR=/tmp
echo "== b64 tests (shipped)" && timeout -k 10 300 python -u -m pytest tests/test_gpu_b64.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r06c2/pytest_b64_shipped.txt 2>&1 && tail -2 gpurun_out/r06c2/pytest_b64_shipped.txt &&
echo "== b64 tests (win64)" && LBF_LIB=$PWD/bitflood_amd/lib/ab_win64/liblbfhash.so timeout -k 10 300 python -u -m pytest tests/test_gpu_b64.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r06c2/pytest_b64_win64.txt 2>&1 && tail -2 gpurun_out/r06c2/pytest_b64_win64.txt &&
echo "== fuzz win64" && LBF_LIB=$PWD/bitflood_amd/lib/ab_win64/liblbfhash.so timeout -k 10 120 python -u tools/fuzz_b64.py --seconds 40 --seed 606 > gpurun_out/r06c2/fuzz_b64_win64.txt 2>&1 && tail -2 gpurun_out/r06c2/fuzz_b64_win64.txt &&
echo "== ab traces" && bash tools/b64_ab_trace.sh r06_win64 3 shipped win64 > gpurun_out/r06c2/ab_trace.log 2>&1 && tail -3 gpurun_out/r06c2/ab_trace.log &&
echo "== register cost" && timeout -k 10 400 python -u tools/register_cost.py > gpurun_out/r06c2/register_cost.json 2> gpurun_out/r06c2/register_cost.err && tail -c 600 gpurun_out/r06c2/register_cost.json
