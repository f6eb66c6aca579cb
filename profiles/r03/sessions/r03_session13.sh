#!/bin/bash
# Round-3 GPU session 13: the new pc4x2 kernel (variant 12; two pc4 groups per
# 6-wave workgroup, producers two to a SIMD): parity tests over every shipped
# variant, a variant sweep against pcx5 (10) and pc4 (7), then a kernel fuzz.
set -o pipefail
O=gpurun_out/r03/s13
mkdir -p $O
T="timeout -k 10"
$T 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_parity.txt 2>&1 &&
$T 300 python -u tools/sweep_variants.py --variants 7,10,12 --max-gib 32 --reps 3 > $O/sweep_7_10_12.jsonl 2> $O/sweep.err &&
$T 150 python -u tools/fuzz_gpu.py --seconds 90 --seed 1301 > $O/fuzz_gpu.txt 2>&1
