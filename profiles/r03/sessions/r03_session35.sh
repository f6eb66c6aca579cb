#!/bin/bash
# Round-3 GPU session 35: pc4 with both producers at wave priority 1, 2, 3
# (31, 32, 33) against the shipped kernel (7), alternating, forward then
# reverse order, at C2 and 16 K x 1 MiB.
set -o pipefail
O=gpurun_out/r03/s35
mkdir -p $O
T="timeout -k 10"
export LBF_LIB=bitflood_amd/lib/experimental/liblbfhash.so
$T 250 python -u tools/sweep_variants.py --variants 7,31,32,33,7,31,32,33 --max-gib 32 --reps 5 \
    --points 262144:16384,1048576:16384 > $O/sweep_fwd.jsonl 2> $O/sweep_fwd.err &&
$T 250 python -u tools/sweep_variants.py --variants 33,32,31,7,33,32,31,7 --max-gib 32 --reps 5 \
    --points 262144:16384,1048576:16384 > $O/sweep_rev.jsonl 2> $O/sweep_rev.err
