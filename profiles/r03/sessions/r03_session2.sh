#!/bin/bash
# Round-3 GPU session 2: the 8-rank C4 rehearsal launched by bench.py itself
# (8 ranks on the one GPU, gloo), the default bench, and the round's C2
# rocprofv3 evidence (trace + PMC passes, tools/profile_round.sh).
set -o pipefail
O=gpurun_out/r03/s2
mkdir -p $O
T="timeout -k 10"
$T 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_bench_ranks.py -m gpu > $O/pytest_bench_ranks.txt 2>&1 &&
LBF_BENCH_BACKEND=gloo $T 600 python -u bench.py --gpus 8 --config c4 > $O/bench_c4_n8_spawned.json 2> $O/bench_c4_n8_spawned.err &&
$T 300 python -u bench.py > $O/bench_c2_n1.json 2> $O/bench_c2_n1.err &&
bash tools/profile_round.sh c2_r03 > $O/profile_c2.txt 2>&1 &&
# host ASan/UBSan over the C ABI with the many-file windows forced small
# (LBF_FILES_WINDOW=2: every multi-file verify job runs in windows)
bash tools/asan_build.sh > $O/asan_build.txt 2>&1 &&
mkdir -p /tmp/asan_scratch &&
LBF_FILES_WINDOW=2 ASAN_OPTIONS=detect_leaks=0 $T 200 tools/build/asan/asan_capi /tmp/asan_scratch 90 93 > $O/asan_windows_seed93.txt 2>&1
