#!/bin/bash
# Round 6, last tree (the flood-file reader changed after tools/r06_final.sh):
# the -m gpu suite, smoke() and the default bench line.
set -o pipefail
out=gpurun_out/r06final2; mkdir -p $out
export TMPDIR=/tmp
echo "== pytest -m gpu" && timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rP --durations=15 --timeout 300 --timeout-method thread -p no:cacheprovider > $out/pytest_gpu.txt 2>&1 && tail -3 $out/pytest_gpu.txt &&
echo "== smoke" && timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1 && tail -2 $out/smoke.txt &&
echo "== bench N=1" && timeout -k 10 400 python bench.py > $out/bench_c2.json 2> $out/bench_c2.err && tail -c 300 $out/bench_c2.json
