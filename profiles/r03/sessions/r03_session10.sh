#!/bin/bash
# Round-3 GPU session 10: after the staging copy helpers became per-worker
# (CopyPool, a host-path change): the whole -m gpu suite, smoke(), the default bench.
set -o pipefail
O=gpurun_out/r03/s10
mkdir -p $O
T="timeout -k 10"
$T 900 python -u -m pytest tests -m gpu -v -rP --durations=15 --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.txt 2>&1 &&
$T 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 &&
$T 300 python -u bench.py --steps 20 --warmup 5 > $O/bench_c2_n1.json 2> $O/bench_c2_n1.err
