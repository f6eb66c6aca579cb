#!/bin/bash
# Round 6: host sanitizers over the C ABI stress driver (tools/asan_capi.cpp,
# now with gap-free tables and a second context registering inside a job's
# on-the-fly pages), and the host-path fuzzer with on-the-fly pinning forced on.
set -o pipefail
out=gpurun_out/r06san; mkdir -p $out
export TMPDIR=/tmp
scratch=$(mktemp -d)
bash tools/asan_build.sh > $out/asan_build.txt 2>&1 && bash tools/tsan_build.sh > $out/tsan_build.txt 2>&1 &&
echo "== asan" && ASAN_OPTIONS=detect_leaks=0 timeout -k 10 200 tools/build/asan/asan_capi $scratch 90 61 > $out/asan_capi.txt 2>&1 && tail -2 $out/asan_capi.txt &&
echo "== tsan" && TSAN_OPTIONS="halt_on_error=1 report_signal_unsafe=0 suppressions=tools/tsan.supp" timeout -k 10 300 tools/build/tsan/tsan_capi $scratch 120 62 > $out/tsan_capi.txt 2>&1 && tail -2 $out/tsan_capi.txt &&
echo "== fuzz host paths, on-the-fly pinning on" && LBF_AUTOPIN=1 LBF_AUTOPIN_MIN_MB=1 LBF_COPY_THREADS=3 timeout -k 10 150 python -u tools/fuzz_host_paths.py --seconds 90 --seed 63 > $out/fuzz_host_paths_autopin.txt 2>&1 && tail -2 $out/fuzz_host_paths_autopin.txt
rc=$?; rm -rf $scratch; exit $rc
