#!/bin/bash
# Round-3 GPU session 4: the leecher's verify/write split and adaptive batch
# deadline -- the C++ GPU tests (C5 16 GiB included), then the 16 GiB
# deadline sweep and the reference's one-request shape.
set -o pipefail
O=gpurun_out/r03/s4
mkdir -p $O
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_host_cpp.py -m gpu -v -rP --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_host_cpp.txt 2>&1 &&
for d in 0 2 10 50; do
  $T 300 bitflood_amd/lib/lbf_loopback --size 17179869184 --chunksize 262144 --window 4096 --batch 1024 \
      --corrupt 1000 --synthetic --threads 16 --deadline-ms $d --dir /tmp/c5_$d > $O/c5_deadline_$d.json 2> $O/c5_deadline_$d.err || exit 1
done &&
$T 300 bitflood_amd/lib/lbf_loopback --size 268435456 --chunksize 262144 --window 1 --batch 1 --deadline-ms 0 \
    --synthetic --threads 16 --dir /tmp/c5_ref > $O/c5_reference_shape_256mib.json 2> $O/c5_reference_shape.err
