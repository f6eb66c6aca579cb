#!/bin/bash
# Round-3 GPU session 15: is pc4x2's per-step cost its structure (3-slot ring,
# six-step loop, prologue barrier) or the second group?  Experimental variant 13
# runs that structure with ONE group per CU at C2's 16 K chains, against pc4 (7).
set -o pipefail
O=gpurun_out/r03/s15c
mkdir -p $O
T="timeout -k 10"
for k in 1 2; do
  LBF_LIB=bitflood_amd/lib/experimental/liblbfhash.so $T 200 python -u tools/sweep_variants.py --variants 7,16,13 --max-gib 32 --reps 5 \
      --points 262144:16384,1048576:16384,262144:32768 > $O/sweep_7_16_13_$k.jsonl 2> $O/sweep_$k.err || exit 1
done
