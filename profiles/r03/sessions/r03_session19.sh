#!/bin/bash
# Round-3 GPU session 19: scheduling barriers around pc4x2's producer barrier
# (18; one-group form 19) against pc4x2 (12), its one-group form (13) and pc4 (7).
set -o pipefail
O=gpurun_out/r03/s19
mkdir -p $O
T="timeout -k 10"
for k in 1 2; do
  LBF_LIB=bitflood_amd/lib/experimental/liblbfhash.so $T 250 python -u tools/sweep_variants.py --variants 7,13,19,12,18 --max-gib 32 --reps 5 \
      --points 262144:16384,1048576:16384,262144:32768,1048576:32768 > $O/sweep_$k.jsonl 2> $O/sweep_$k.err || exit 1
done
