#!/bin/bash
# Round-3 GPU session 34: pc4 producer priorities (producer 0, producer 1) --
# 7 (0, 0, the shipped kernel), 29 (0, 1), 30 (1, 0), 31 (1, 1) -- alternating,
# forward then reverse order, at C2 and 16 K x 1 MiB.
set -o pipefail
O=gpurun_out/r03/s34
mkdir -p $O
T="timeout -k 10"
export LBF_LIB=bitflood_amd/lib/experimental/liblbfhash.so
$T 250 python -u tools/sweep_variants.py --variants 7,29,30,31,7,29,30,31 --max-gib 32 --reps 5 \
    --points 262144:16384,1048576:16384 > $O/sweep_fwd.jsonl 2> $O/sweep_fwd.err &&
$T 250 python -u tools/sweep_variants.py --variants 31,30,29,7,31,30,29,7 --max-gib 32 --reps 5 \
    --points 262144:16384,1048576:16384 > $O/sweep_rev.jsonl 2> $O/sweep_rev.err
