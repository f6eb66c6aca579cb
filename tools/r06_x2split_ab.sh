#!/bin/bash
# Round 6 A/B at C4: pc4x2 (variant 12, shipped) against one group per
# workgroup, two workgroups per CU (experimental 38/39): parity, then timings.
set -o pipefail
out=gpurun_out/r06x2split; mkdir -p $out
export TMPDIR=/tmp
LIB=$PWD/tools/build/experimental/liblbfhash.so
make -C tools/experimental > $out/build.txt 2>&1 &&
echo "== fuzz 38,39" && LBF_LIB=$LIB LBF_FUZZ_VARIANTS=38,39 timeout -k 10 120 python -u tools/fuzz_gpu.py --seconds 40 --seed 638 > $out/fuzz.txt 2>&1 && tail -1 $out/fuzz.txt | cut -c1-200 &&
echo "== sweep" && LBF_LIB=$LIB timeout -k 10 400 python -u tools/sweep_variants.py --max-gib 32 --reps 5 --variants 12,38,39,12,38,39 \
  --points 1048576:32768,262144:32768,262144:24576 > $out/sweep.jsonl 2>&1; rc=$?; cut -c1-170 $out/sweep.jsonl; exit $rc
