#!/bin/bash
# Round-3 GPU session 16: (a) stamps of pc4 (7) vs pc4x2's structure with one
# group (13); (b) 13 with pc4's LDS layout (17); (c) pc4's fast loop unrolled
# by 8 (16) against 4 (7) at C2, alternating, 20 reps each.
set -o pipefail
O=gpurun_out/r03/s16
mkdir -p $O
T="timeout -k 10"
$T 200 tools/build/probe_pc > $O/probe_pc_x1.log 2>&1 &&
LBF_LIB=bitflood_amd/lib/experimental/liblbfhash.so $T 200 python -u tools/sweep_variants.py --variants 7,13,17 --max-gib 16 --reps 5 \
    --points 262144:16384,1048576:16384 > $O/sweep_7_13_17.jsonl 2> $O/sweep_a.err &&
LBF_LIB=bitflood_amd/lib/experimental/liblbfhash.so $T 300 python -u tools/sweep_variants.py --variants 7,16,7,16,7,16 --max-gib 4 --reps 20 \
    --points 262144:16384 > $O/sweep_7_16_c2.jsonl 2> $O/sweep_b.err
