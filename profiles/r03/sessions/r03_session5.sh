#!/bin/bash
# Round-3 GPU session 5: ThreadSanitizer over the C5 harness after the
# leecher's verify/write split (reader, decode, verifier, writer and sender
# threads of both peers), and over the C++ layer's GPU tests (ReceiveChunks =
# VerifyChunks + WriteChunks).  Host code instrumented only.
set -o pipefail
O=gpurun_out/r03/s5
mkdir -p $O
T="timeout -k 10"
export TSAN_OPTIONS="halt_on_error=1 report_signal_unsafe=0 suppressions=tools/tsan.supp"
bash tools/tsan_build.sh > $O/tsan_build.txt 2>&1 &&
mkdir -p /tmp/tsan_scratch &&
$T 300 tools/build/tsan/tsan_gpu_tests /tmp/tsan_scratch > $O/tsan_gpu_tests.txt 2>&1 &&
$T 300 tools/build/tsan/tsan_loopback --size 67108864 --chunksize 262144 --window 64 --batch 16 --corrupt 7 \
    --threads 8 --dir /tmp/tsan_l1 > $O/tsan_loopback.txt 2>&1 &&
$T 300 tools/build/tsan/tsan_loopback --size 16789561 --chunksize 65539 --window 512 --batch 128 --corrupt 5 \
    --threads 8 --synthetic --deadline-ms 2 --dir /tmp/tsan_l2 >> $O/tsan_loopback.txt 2>&1 &&
$T 300 tools/build/tsan/tsan_loopback --size 33554432 --chunksize 262144 --window 256 --batch 64 --threads 8 \
    --no-register --deadline-ms 0 --dir /tmp/tsan_l3 >> $O/tsan_loopback.txt 2>&1
