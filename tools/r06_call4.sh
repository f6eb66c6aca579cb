set -o pipefail
mkdir -p gpurun_out/r06c4
export TMPDIR=/tmp
echo "== registered tests" && timeout -k 10 400 python -u -m pytest tests/test_gpu_registered.py tests/test_gpu_workers.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r06c4/pytest_registered.txt 2>&1 && tail -2 gpurun_out/r06c4/pytest_registered.txt &&
for k in thp numpy 4k; do
  echo "== register cost $k" && timeout -k 10 300 python -u tools/register_cost.py --kind $k --sizes 64,1024,4096 > gpurun_out/r06c4/register_cost_$k.json 2> gpurun_out/r06c4/register_cost_$k.err || exit 1
  tail -c 300 gpurun_out/r06c4/register_cost_$k.json
done
