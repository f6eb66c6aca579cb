#!/bin/bash
# Round-3 GPU session 17: pc4x2 with its stores paired again (slot offset
# laundered through an empty asm): parity over every shipped variant, then
# pc4 (7), one-group pc4x2 (13), pcx5 (10) and pc4x2 (12), two sweeps.
set -o pipefail
O=gpurun_out/r03/s17
mkdir -p $O
T="timeout -k 10"
$T 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_parity.txt 2>&1 &&
for k in 1 2; do
  LBF_LIB=bitflood_amd/lib/experimental/liblbfhash.so $T 250 python -u tools/sweep_variants.py --variants 7,13,10,12 --max-gib 32 --reps 5 \
      --points 262144:16384,1048576:16384,262144:20000,262144:32768,1048576:32768 > $O/sweep_$k.jsonl 2> $O/sweep_$k.err || exit 1
done
