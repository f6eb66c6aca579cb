#!/bin/bash
# Round-3 GPU session 1: new tests, the self-launched multi-rank bench
# rehearsals and the C5 deadline sweep.  Every GPU step has its own time limit
# and the steps are chained with && (a failure ends the session).
set -o pipefail
O=gpurun_out/r03/s1
mkdir -p $O
T="timeout -k 10"
{ [ -n "$SKIP_PYTEST" ] || $T 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_files.py "tests/test_host_cpp.py::test_encoder_cli_file_past_4gib" \
    tests/test_gpu_parity.py tests/test_gpu_registered.py -m gpu > $O/pytest_new.log 2>&1; } &&
$T 300 python -u bench.py > $O/bench_c2_n1.json 2> $O/bench_c2_n1.err &&
LBF_BENCH_BACKEND=gloo $T 300 python -u bench.py --gpus 2 > $O/bench_c2_n2_spawned.json 2> $O/bench_c2_n2_spawned.err &&
LBF_WORKERS_PER_DEVICE=2 $T 300 python -u bench.py --gpus 2 > $O/bench_c2_n2_spawned_w2.json 2> $O/bench_c2_n2_spawned_w2.err &&
for d in 0 2 10 50; do
  $T 300 bitflood_amd/lib/lbf_loopback --size 17179869184 --chunksize 262144 --window 4096 --batch 1024 \
      --corrupt 1000 --synthetic --threads 16 --deadline-ms $d --dir /tmp/c5_$d > $O/c5_deadline_$d.json 2> $O/c5_deadline_$d.err || exit 1
done &&
$T 300 bitflood_amd/lib/lbf_loopback --size 268435456 --chunksize 262144 --window 1 --batch 1 --deadline-ms 0 \
    --synthetic --threads 16 --dir /tmp/c5_ref > $O/c5_reference_shape_256mib.json 2> $O/c5_reference_shape.err
