#!/bin/bash
# Round 6: where pc4x2's extra cycles per step go: the
# stamped diagnostic build (s_memtime around every barrier), per role and,
# for pc4x2, per consumer wave.
set -o pipefail
out=gpurun_out/r06stamps; mkdir -p $out tools/build
cd tools && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -DLBF_PC_STAMPS -I../include -I../bitflood_amd/csrc \
  probe_pc.hip -o build/probe_pc -L/opt/rocm/lib -lhsa-runtime64 > ../$out/build.txt 2>&1 && cd .. &&
timeout -k 10 180 tools/build/probe_pc > $out/probe_pc.txt 2>&1; rc=$?; cat $out/probe_pc.txt; exit $rc
