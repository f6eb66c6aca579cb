#!/bin/bash
# tools/asan_build.sh -- build tools/build/asan/asan_capi: the C ABI (kernels +
# lbf_capi.cpp) and the stress driver with AddressSanitizer + UBSan on the HOST
# code only (-Xarch_host before each -fsanitize; the gfx950 device code is not
# instrumented), plus the oracle as the checker.  Run on the GPU box:
#   ASAN_OPTIONS=detect_leaks=0 tools/build/asan/asan_capi <scratch> [seconds] [seed]
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=tools/build/asan
mkdir -p "$OUT"
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
SAN="-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-omit-frame-pointer"
FLAGS="--offload-arch=gfx950 -O1 -g -std=c++17 -fPIC -Iinclude -Ibitflood_amd/csrc $SAN"
$HIPCC $FLAGS -c -o $OUT/sha1_kernels.o bitflood_amd/csrc/sha1_kernels.hip
$HIPCC $FLAGS -x hip -c -o $OUT/lbf_capi.o bitflood_amd/csrc/lbf_capi.cpp
$HIPCC $FLAGS -c -o $OUT/asan_capi.o tools/asan_capi.cpp
# the oracle is the checker, not under test: plain -O2
gcc -O2 -fPIC -c -o $OUT/sha1_oracle.o oracle/sha1_oracle.c -Ioracle
$HIPCC --offload-arch=gfx950 $SAN -o $OUT/asan_capi $OUT/asan_capi.o $OUT/lbf_capi.o $OUT/sha1_kernels.o \
  $OUT/sha1_oracle.o -lpthread -L/opt/rocm/lib -lhsa-runtime64
echo "built $OUT/asan_capi"
