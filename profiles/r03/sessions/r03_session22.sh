#!/bin/bash
# Round-3 GPU session 22: pc4x2 split into a shipped kernel and diagnostic
# wrappers around one body -- parity, then its six-step loop (12) against
# twelve steps (21), alternating.
set -o pipefail
O=gpurun_out/r03/s22
mkdir -p $O
T="timeout -k 10"
$T 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_parity.txt 2>&1 &&
for k in 1 2; do
  LBF_LIB=bitflood_amd/lib/experimental/liblbfhash.so $T 250 python -u tools/sweep_variants.py --variants 12,21,12,21 --max-gib 32 --reps 5 \
      --points 262144:32768,1048576:32768,262144:24576 > $O/sweep_$k.jsonl 2> $O/sweep_$k.err || exit 1
done
