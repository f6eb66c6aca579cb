#!/bin/bash
# Round-3 GPU session 12: bench.py after its host-memory leg became
# failure-tolerant -- the default N=1 line and a self-launched 2-rank run.
set -o pipefail
O=gpurun_out/r03/s12
mkdir -p $O
T="timeout -k 10"
$T 300 python -u bench.py > $O/bench_c2_n1.json 2> $O/bench_c2_n1.err &&
$T 300 python -u bench.py --gpus 2 --steps 5 --warmup 2 > $O/bench_c2_n2_spawned.json 2> $O/bench_c2_n2_spawned.err
