#!/bin/bash
# Round-3 GPU session 30 (after the pc4x2 consumer priority), the round's final tree on one box: what the driver
# runs at round end (-m gpu suite, smoke(), default bench.py), the N-rank flow
# (self-launched and under torch.distributed.run), rocprofv3 evidence of C2 and
# C4, and kernel + host-path fuzz passes against the oracle.
set -o pipefail
O=gpurun_out/r03/s30
mkdir -p $O
T="timeout -k 10"
$T 900 python -u -m pytest tests -m gpu -v -rP --durations=15 --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.txt 2>&1 &&
$T 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 &&
$T 300 python -u bench.py > $O/bench_c2_n1.json 2> $O/bench_c2_n1.err &&
$T 300 python -u bench.py --gpus 2 --steps 5 --warmup 2 > $O/bench_c2_n2_spawned.json 2> $O/bench_c2_n2_spawned.err &&
LBF_BENCH_BACKEND=gloo $T 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29547 bench.py --gpus 2 --steps 5 --warmup 2 > $O/bench_c2_n2_torchrun.json 2> $O/bench_c2_n2_torchrun.err &&
bash tools/profile_round.sh c2_r03d > $O/profile_c2.txt 2>&1 &&
bash tools/profile_round.sh c4_r03d --config c4 --no-e2e --no-cpu-baseline > $O/profile_c4.txt 2>&1 &&
$T 150 python -u tools/fuzz_gpu.py --seconds 90 --seed 3001 > $O/fuzz_gpu.txt 2>&1 &&
LBF_COPY_THREADS=8 $T 120 python -u tools/fuzz_host_paths.py --seconds 60 --seed 3002 > $O/fuzz_host_paths.txt 2>&1
