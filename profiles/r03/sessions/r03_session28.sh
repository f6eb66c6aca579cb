#!/bin/bash
# Round-3 GPU session 28: consumers at wave priority 3 (s_setprio) in pc4x2 (22)
# and its one-group form (23), against 12, 13 and pc4 (7), alternating.
set -o pipefail
O=gpurun_out/r03/s28
mkdir -p $O
T="timeout -k 10"
for k in 1 2; do
  LBF_LIB=bitflood_amd/lib/experimental/liblbfhash.so $T 250 python -u tools/sweep_variants.py --variants 7,13,23,12,22 --max-gib 32 --reps 5 \
      --points 262144:16384,1048576:16384,1048576:32768 > $O/sweep_$k.jsonl 2> $O/sweep_$k.err || exit 1
done
