#!/bin/bash
# Round-3 GPU session 33: pc4x2 producer priorities (group 0, group 1) --
# 25 (0, 1, the shipped code), 26 (1, 0), 27 (0, 2), 28 (1, 2) -- alternating,
# forward then reverse order, at C4 shapes.
set -o pipefail
O=gpurun_out/r03/s33
mkdir -p $O
T="timeout -k 10"
export LBF_LIB=bitflood_amd/lib/experimental/liblbfhash.so
$T 250 python -u tools/sweep_variants.py --variants 25,26,27,28,25,26,27,28 --max-gib 32 --reps 5 \
    --points 1048576:32768,262144:24576 > $O/sweep_fwd.jsonl 2> $O/sweep_fwd.err &&
$T 250 python -u tools/sweep_variants.py --variants 28,27,26,25,28,27,26,25 --max-gib 32 --reps 5 \
    --points 1048576:32768,262144:24576 > $O/sweep_rev.jsonl 2> $O/sweep_rev.err
