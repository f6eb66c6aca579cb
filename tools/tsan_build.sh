#!/bin/bash
# tools/tsan_build.sh -- build tools/build/tsan/tsan_capi: the C ABI (kernels +
# lbf_capi.cpp) and the stress driver of tools/asan_capi.cpp with
# ThreadSanitizer on the HOST code only (-Xarch_host before -fsanitize; the
# gfx950 device code is not instrumented), plus the oracle as the checker.
# The driver's contexts run 1-4 workers, each with its own host thread and
# staging-copy helper threads, so the races it can find are the host
# pipeline's own.  Run on the GPU box:
#   TSAN_OPTIONS="halt_on_error=1 report_signal_unsafe=0 suppressions=tools/tsan.supp" \
#     tools/build/tsan/tsan_capi <scratch> [seconds] [seed]
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=tools/build/tsan
mkdir -p "$OUT"
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
SAN="-Xarch_host -fsanitize=thread -Xarch_host -fno-omit-frame-pointer"
FLAGS="--offload-arch=gfx950 -O1 -g -std=c++17 -fPIC -Iinclude -Ibitflood_amd/csrc $SAN"
$HIPCC $FLAGS -c -o $OUT/sha1_kernels.o bitflood_amd/csrc/sha1_kernels.hip
$HIPCC $FLAGS -x hip -c -o $OUT/lbf_capi.o bitflood_amd/csrc/lbf_capi.cpp
$HIPCC $FLAGS -c -o $OUT/tsan_capi.o tools/asan_capi.cpp
gcc -O2 -fPIC -c -o $OUT/sha1_oracle.o oracle/sha1_oracle.c -Ioracle
$HIPCC --offload-arch=gfx950 $SAN -o $OUT/tsan_capi $OUT/tsan_capi.o $OUT/lbf_capi.o $OUT/sha1_kernels.o \
  $OUT/sha1_oracle.o -lpthread -L/opt/rocm/lib -lhsa-runtime64
echo "built $OUT/tsan_capi"
# the C++ libBitFlood layer and its GPU test program (8 threads on Base64Encode,
# SetDeviceMask under 4 hashing threads, the Flood verify paths) on the same
# instrumented C ABI:  tools/build/tsan/tsan_gpu_tests <scratch>
for f in Encoder FloodFile Flood PeerWire gpu_tests; do
  $HIPCC -O1 -g -std=c++17 -fPIC -Iinclude $SAN -c -o $OUT/$f.o bitflood_amd/host/$f.cpp
done
$HIPCC --offload-arch=gfx950 $SAN -o $OUT/tsan_gpu_tests $OUT/gpu_tests.o $OUT/Encoder.o $OUT/FloodFile.o \
  $OUT/Flood.o $OUT/PeerWire.o $OUT/lbf_capi.o $OUT/sha1_kernels.o -lpthread -L/opt/rocm/lib -lhsa-runtime64
echo "built $OUT/tsan_gpu_tests"
# the C5 harness (reader, decode, verifier and sender threads of two peers):
#   tools/build/tsan/tsan_loopback --size N --dir <scratch> ...
$HIPCC -O1 -g -std=c++17 -fPIC -Iinclude $SAN -c -o $OUT/lbf_loopback.o bitflood_amd/host/lbf_loopback.cpp
$HIPCC --offload-arch=gfx950 $SAN -o $OUT/tsan_loopback $OUT/lbf_loopback.o $OUT/Encoder.o $OUT/FloodFile.o \
  $OUT/Flood.o $OUT/PeerWire.o $OUT/lbf_capi.o $OUT/sha1_kernels.o -lpthread -L/opt/rocm/lib -lhsa-runtime64
echo "built $OUT/tsan_loopback"
