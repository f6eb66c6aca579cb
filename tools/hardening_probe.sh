# GPU-box check after host-side changes to lbf_capi.cpp: the host-path GPU tests
# (parity, workers, concurrency, C++ suite) and one host-ASAN stress run.
set -o pipefail
out=gpurun_out/hardening
mkdir -p $out
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py tests/test_gpu_workers.py tests/test_gpu_concurrency.py tests/test_host_cpp.py -m gpu \
  > $out/pytest.log 2>&1 &&
ASAN_OPTIONS=detect_leaks=0 timeout -k 10 200 tools/build/asan/asan_capi /tmp/asan_scratch 90 31 > $out/asan_seed31.log 2>&1
