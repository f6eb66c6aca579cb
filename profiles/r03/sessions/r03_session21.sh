#!/bin/bash
# Round-3 GPU session 21: pc4's fast loop written as a compile-time loop (the
# shipped eight steps, 7) against four (16) and sixteen (20) steps at C2,
# alternating, 20 reps each, after the parity tests.
set -o pipefail
O=gpurun_out/r03/s21
mkdir -p $O
T="timeout -k 10"
$T 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_parity.txt 2>&1 &&
for k in 1 2; do
  LBF_LIB=bitflood_amd/lib/experimental/liblbfhash.so $T 250 python -u tools/sweep_variants.py --variants 16,7,20,16,7,20 --max-gib 16 --reps 20 \
      --points 262144:16384,1048576:16384 > $O/sweep_$k.jsonl 2> $O/sweep_$k.err || exit 1
done
