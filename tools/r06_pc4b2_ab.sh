#!/bin/bash
# Round 6 A/B: pc4 (variant 7, shipped) against variant 37 (one barrier per two
# steps, tools/experimental/), built on the box.  Parity first (fuzz against the
# oracle, digests equal to variant 7's), then alternating timings.
set -o pipefail
out=gpurun_out/r06pc4b2; mkdir -p $out
export TMPDIR=/tmp
LIB=$PWD/tools/build/experimental/liblbfhash.so
make -C tools/experimental > $out/build.txt 2>&1 &&
echo "== fuzz 37" && LBF_LIB=$LIB LBF_FUZZ_VARIANTS=37 timeout -k 10 120 python -u tools/fuzz_gpu.py --seconds 60 --seed 637 > $out/fuzz_37.txt 2>&1 && tail -1 $out/fuzz_37.txt &&
echo "== sweep" && LBF_LIB=$LIB timeout -k 10 300 python -u tools/sweep_variants.py --max-gib 16 --reps 10 --variants 7,37,7,37,7,37 \
  --points 262144:16384,262144:8192,1048576:16384,65536:16384 > $out/sweep.jsonl 2>&1 && cat $out/sweep.jsonl | cut -c1-160 &&
echo "== bench A/B" && for r in 1 2 3; do for v in 7 37; do
  LBF_LIB=$LIB timeout -k 10 200 python -u bench.py --variant $v --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-other-configs > $out/bench_v${v}_$r.json 2> $out/bench_v${v}_$r.err || exit 1
  python3 -c "import json,sys; d=json.loads(open('$out/bench_v${v}_$r.json').read().strip().splitlines()[-1]); print($v, $r, d['ms_per_step'], d['value'], d['parity']['per_rank'])"
done; done
