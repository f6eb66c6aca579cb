#!/bin/bash
# Round-3 GPU session 36: what the driver runs at round end, on the tree as
# committed last (-m gpu suite, smoke(), default bench).
set -o pipefail
O=gpurun_out/r03/s36
mkdir -p $O
T="timeout -k 10"
$T 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.txt 2>&1 &&
$T 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 &&
$T 300 python -u bench.py > $O/bench_c2_n1.json 2> $O/bench_c2_n1.err
