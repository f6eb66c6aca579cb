#!/bin/bash
# Round-3 GPU session 3: the whole -m gpu suite on the round's final code, the
# driver's smoke(), and a torchrun-launched 2-rank rehearsal (the launcher
# path the driver's scaling run uses), each step under its own time limit.
set -o pipefail
O=gpurun_out/r03/s3
mkdir -p $O
T="timeout -k 10"
$T 900 python -u -m pytest tests -m gpu -v -rP --durations=15 --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.txt 2>&1 &&
$T 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 &&
LBF_BENCH_BACKEND=gloo $T 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 > $O/bench_c2_n2_torchrun.json 2> $O/bench_c2_n2_torchrun.err
