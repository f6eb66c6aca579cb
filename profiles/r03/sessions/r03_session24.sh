#!/bin/bash
# Round-3 GPU session 24: bench.py's N-rank flow after dist_setup moved the
# process-group set-up behind a stdout -> stderr redirect: torchrun and
# self-launched 2-rank runs must leave exactly one JSON line on stdout.
set -o pipefail
O=gpurun_out/r03/s24
mkdir -p $O
T="timeout -k 10"
LBF_BENCH_BACKEND=gloo $T 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29543 bench.py --gpus 2 --steps 5 --warmup 2 > $O/bench_c2_n2_torchrun.json 2> $O/bench_c2_n2_torchrun.err &&
$T 300 python -u bench.py --gpus 2 --steps 5 --warmup 2 > $O/bench_c2_n2_spawned.json 2> $O/bench_c2_n2_spawned.err &&
python -c "
import json
for f in ['$O/bench_c2_n2_torchrun.json', '$O/bench_c2_n2_spawned.json']:
    lines = [l for l in open(f) if l.strip()]
    assert len(lines) == 1, (f, len(lines))
    d = json.loads(lines[0])
    print(f, d['n_gpus'], d['parity']['per_rank'], d['e2e']['parity_per_rank'], d['e2e']['failed_per_rank'])
" > $O/check.txt 2>&1
