#!/bin/bash
# Round-3 GPU session 14: where pc4x2's consumer loses its ~150 cycles per step
# (stamped builds: group 1 idle at the barriers / producers without LDS stores),
# and pcx5 (10) against pc4x2 (12) between 16 K and 32 K chains, twice.
set -o pipefail
O=gpurun_out/r03/s14
mkdir -p $O
T="timeout -k 10"
$T 100 tools/build/probe_pc_x2diag1 > $O/x2diag1_group1_idle.log 2>&1 &&
$T 100 tools/build/probe_pc_x2diag2 > $O/x2diag2_no_stores.log 2>&1 &&
for k in 1 2; do
  $T 200 python -u tools/sweep_variants.py --variants 10,12 --max-gib 32 --reps 5 \
      --points 262144:20000,262144:24576,262144:28672,262144:32768,1048576:20000,1048576:24576,1048576:32768 \
      > $O/sweep_10_12_$k.jsonl 2> $O/sweep_$k.err || exit 1
done
