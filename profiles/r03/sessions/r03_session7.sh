#!/bin/bash
# Round-3 GPU session 7: randomised checks on the round's host-side changes --
# the host-path fuzzer with its new multi-file mode (random LBF_FILES_WINDOW),
# at 3 and 8 copy threads, and the CLI fuzzer (lbf_encoder / lbf_verify with
# the reference-form size attribute) -- everything against the oracle/hashlib.
set -o pipefail
O=gpurun_out/r03/s7
mkdir -p $O
T="timeout -k 10"
LBF_COPY_THREADS=3 $T 200 python -u tools/fuzz_host_paths.py --seconds 120 --seed 301 > $O/fuzz_host_paths_t3.txt 2>&1 &&
LBF_COPY_THREADS=8 $T 200 python -u tools/fuzz_host_paths.py --seconds 120 --seed 302 > $O/fuzz_host_paths_t8.txt 2>&1 &&
$T 200 python -u tools/fuzz_cli.py --seconds 120 --seed 303 > $O/fuzz_cli.txt 2>&1
