#!/bin/bash
# Round-3 GPU session 18: the round's final kernels (pc4 with its eight-step
# loop for C2, pc4x2 for 16-32 K chains): the whole -m gpu suite, smoke(), and
# the rocprofv3 evidence (trace + PMC passes) of the default bench (C2) and of
# bench.py --config c4.
set -o pipefail
O=gpurun_out/r03/s18
mkdir -p $O
T="timeout -k 10"
$T 900 python -u -m pytest tests -m gpu -v -rP --durations=15 --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.txt 2>&1 &&
$T 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 &&
bash tools/profile_round.sh c2_r03b > $O/profile_c2.txt 2>&1 &&
bash tools/profile_round.sh c4_r03 --config c4 --no-e2e --no-cpu-baseline > $O/profile_c4.txt 2>&1
