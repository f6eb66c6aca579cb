set -o pipefail
mkdir -p gpurun_out/cc
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_concurrency.py "tests/test_host_cpp.py::test_cpp_api_gpu_suite" > gpurun_out/cc/pytest.log 2>&1 &&
timeout -k 10 400 env LBF_BENCH_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --config c4 --gpus 2 --steps 3 --warmup 1 --no-e2e > gpurun_out/cc/bench_c4_2rank_gloo.log 2>&1
