#!/bin/bash
# Round 6, final tree: the -m gpu suite, smoke(), the default bench line (the
# driver's N=1 command), then the driver's default 8-GPU command rehearsed on
# the one GPU (bench.py --gpus 8 self-launches eight ranks; they share the
# card, so gloo), its wall time taken against the driver's 600 s limit.
# Each step has its own time limit; the first failure ends the script.
set -o pipefail
out=gpurun_out/r06final; mkdir -p $out
export TMPDIR=/tmp
echo "== pytest -m gpu" && timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rP --durations=15 --timeout 300 --timeout-method thread -p no:cacheprovider > $out/pytest_gpu.txt 2>&1 && tail -3 $out/pytest_gpu.txt &&
echo "== smoke" && timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1 && tail -2 $out/smoke.txt &&
echo "== bench N=1" && timeout -k 10 400 python bench.py > $out/bench_c2.json 2> $out/bench_c2.err && tail -c 400 $out/bench_c2.json &&
echo "== bench --gpus 8 (rehearsal)" && t0=$(date +%s.%N) && timeout -k 10 900 python bench.py --gpus 8 > $out/bench_c2_n8_spawned.json 2> $out/bench_c2_n8_spawned.err; rc=$?; t1=$(date +%s.%N)
echo "{\"command\": \"python bench.py --gpus 8\", \"rc\": $rc, \"wall_s\": $(python3 -c "print(round($t1-$t0,1))"), \"driver_limit_s\": 600}" > $out/bench_c2_n8_wall.json
cat $out/bench_c2_n8_wall.json; tail -c 300 $out/bench_c2_n8_spawned.json; exit $rc
