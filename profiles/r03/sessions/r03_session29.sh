#!/bin/bash
# Round-3 GPU session 29: pc4x2 shipped with its consumers at wave priority 3
# -- parity over every shipped variant, then pc4 (7) against pc4 with its
# consumer at priority 3 (24) at C2, and pc4x2 (12, now with priority) against
# pcx5 (10), alternating.
set -o pipefail
O=gpurun_out/r03/s29
mkdir -p $O
T="timeout -k 10"
$T 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_parity.txt 2>&1 &&
for k in 1 2; do
  LBF_LIB=bitflood_amd/lib/experimental/liblbfhash.so $T 250 python -u tools/sweep_variants.py --variants 7,24,7,24 --max-gib 16 --reps 10 \
      --points 262144:16384,1048576:16384 > $O/sweep_c2_$k.jsonl 2> $O/sweep_c2_$k.err || exit 1
  LBF_LIB=bitflood_amd/lib/experimental/liblbfhash.so $T 250 python -u tools/sweep_variants.py --variants 10,12,10,12 --max-gib 32 --reps 5 \
      --points 262144:20000,262144:24576,262144:32768,1048576:32768 > $O/sweep_c4_$k.jsonl 2> $O/sweep_c4_$k.err || exit 1
done
