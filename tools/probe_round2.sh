#!/bin/bash
# tools/probe_round2.sh -- diagnostics for DESIGN.md (round 2): pcx5 / pc4
# per-role cycle split (s_memtime stamps, tools/probe_pc.hip) and the NUMA A/B
# of the PCIe-inclusive host path (tools/e2e_sizes.py, LBF_NUMA=1/0 twice).
set -o pipefail
out=gpurun_out/probe_r02
mkdir -p "$out"
timeout -k 10 180 tools/build/probe_pc > "$out/probe_pc_stamps.log" 2>&1 && cat "$out/probe_pc_stamps.log" &&
for rep in 1 2; do
  for numa in 1 0; do
    LBF_NUMA=$numa timeout -k 10 240 python tools/e2e_sizes.py > "$out/e2e_numa${numa}_rep${rep}.log" 2>&1 || exit $?
    tail -n 1 "$out/e2e_numa${numa}_rep${rep}.log"
  done
done
