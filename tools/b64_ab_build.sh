#!/bin/bash
# tools/b64_ab_build.sh <name> <defines...> -- an A/B build of the shipped
# library with the wire kernels' geometry changed (e.g. -DLBF_B64_DEC_LINES=72
# -DLBF_B64_DEC_TILES_PER_GROUP=8) into bitflood_amd/lib/ab_<name>/liblbfhash.so,
# for tools/b64_profile.sh <tag> bitflood_amd/lib/ab_<name>/liblbfhash.so.
set -euo pipefail
cd "$(dirname "$0")/../bitflood_amd/csrc"
name=$1; shift
out=../lib/ab_$name
mkdir -p "$out"
flags="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -Wno-unused-value -munsafe-fp-atomics -I../../include -I. $*"
make -s -B OUT="$out" HIPFLAGS="$flags" "$out/liblbfhash.so"
rm -f "$out"/*.o
echo "built $out/liblbfhash.so ($*)"
