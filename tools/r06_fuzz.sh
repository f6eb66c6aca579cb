#!/bin/bash
# Round 6, final tree: a fuzz campaign over every layer against the oracle /
# hashlib / xmlrpc++'s rules; each tool under its own time limit.
set -o pipefail
out=gpurun_out/r06fuzz; mkdir -p $out
export TMPDIR=/tmp
echo "== kernels" && timeout -k 10 200 python -u tools/fuzz_gpu.py --seconds 150 --seed 6601 > $out/fuzz_gpu.txt 2>&1 && tail -1 $out/fuzz_gpu.txt | cut -c1-200 &&
echo "== host paths" && LBF_COPY_THREADS=5 timeout -k 10 180 python -u tools/fuzz_host_paths.py --seconds 120 --seed 6602 > $out/fuzz_host_paths.txt 2>&1 && tail -1 $out/fuzz_host_paths.txt | cut -c1-200 &&
echo "== cli" && timeout -k 10 180 python -u tools/fuzz_cli.py --seconds 120 --seed 6603 > $out/fuzz_cli.txt 2>&1 && tail -1 $out/fuzz_cli.txt | cut -c1-200 &&
echo "== wire" && timeout -k 10 150 python -u tools/fuzz_b64.py --seconds 90 --seed 6604 > $out/fuzz_b64.txt 2>&1 && tail -1 $out/fuzz_b64.txt | cut -c1-200
