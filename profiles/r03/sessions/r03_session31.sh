#!/bin/bash
# Round-3 GPU session 31: pc4x2 (12) against group 1's producers at wave
# priority 1 (25), alternating, at C4 shapes.
set -o pipefail
O=gpurun_out/r03/s31
mkdir -p $O
T="timeout -k 10"
for k in 1 2; do
  LBF_LIB=bitflood_amd/lib/experimental/liblbfhash.so $T 250 python -u tools/sweep_variants.py --variants 12,25,12,25 --max-gib 32 --reps 5 \
      --points 262144:32768,1048576:32768,262144:24576 > $O/sweep_$k.jsonl 2> $O/sweep_$k.err || exit 1
done
