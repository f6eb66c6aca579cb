#!/bin/bash
# Round-3 GPU session 32, the round's final tree after group 1's producers of
# pc4x2 went to wave priority 1 (variant 25 made the shipped variant 12): the
# -m gpu suite, smoke(), the default bench, N=2 self-launched, rocprofv3
# evidence of C4 (C2's pc4 kernel is unchanged), a pcx5 / pc4x2 sweep with the
# shipped library, and a kernel fuzz pass against the oracle.
set -o pipefail
O=gpurun_out/r03/s32
mkdir -p $O
T="timeout -k 10"
$T 900 python -u -m pytest tests -m gpu -v -rP --durations=15 --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.txt 2>&1 &&
$T 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 &&
$T 300 python -u bench.py > $O/bench_c2_n1.json 2> $O/bench_c2_n1.err &&
$T 300 python -u bench.py --gpus 2 --steps 5 --warmup 2 > $O/bench_c2_n2_spawned.json 2> $O/bench_c2_n2_spawned.err &&
bash tools/profile_round.sh c4_r03e --config c4 --no-e2e --no-cpu-baseline > $O/profile_c4.txt 2>&1 &&
$T 250 python -u tools/sweep_variants.py --variants 10,12,10,12 --max-gib 32 --reps 5 \
    --points 1048576:32768,262144:32768,262144:24576,262144:20000 > $O/sweep_10_12.jsonl 2> $O/sweep_10_12.err &&
$T 150 python -u tools/fuzz_gpu.py --seconds 90 --seed 3201 > $O/fuzz_gpu.txt 2>&1
