#!/bin/bash
# Round-3 GPU session 11: sanitizers over the per-worker staging copy helpers
# (CopyPool): the C ABI stress driver under ThreadSanitizer (concurrent callers
# on shared contexts, 24-40 MiB batches, so every worker's pool runs) and under
# ASan/UBSan, and the C++ layer's GPU tests under TSan.  Host code instrumented only.
set -o pipefail
O=gpurun_out/r03/s11
mkdir -p $O
T="timeout -k 10"
export TSAN_OPTIONS="halt_on_error=1 report_signal_unsafe=0 suppressions=tools/tsan.supp"
bash tools/tsan_build.sh > $O/tsan_build.txt 2>&1 &&
mkdir -p /tmp/tsan_scratch /tmp/asan_scratch &&
$T 200 tools/build/tsan/tsan_capi /tmp/tsan_scratch 120 1101 > $O/tsan_capi_seed1101.txt 2>&1 &&
$T 300 tools/build/tsan/tsan_gpu_tests /tmp/tsan_scratch > $O/tsan_gpu_tests.txt 2>&1 &&
bash tools/asan_build.sh > $O/asan_build.txt 2>&1 &&
ASAN_OPTIONS=detect_leaks=0 $T 200 tools/build/asan/asan_capi /tmp/asan_scratch 90 1102 > $O/asan_capi_seed1102.txt 2>&1
