#!/bin/bash
# Round-3 GPU session 9 (after CopyPool): is C3's slow first EncodeFile a first read of freshly
# written tmpfs pages (kernel side) or ours?  Three fresh 64 x 1 GiB sets:
# host pread first; our in-process batch first; the CLI first with 16 copy threads.
set -o pipefail
O=gpurun_out/r03/s9
mkdir -p $O
T="timeout -k 10"
$T 300 python -u tools/c3_e2e_probe.py --order pread,cli --skip inproc > $O/pread_first.jsonl 2> $O/pread_first.err &&
$T 300 python -u tools/c3_e2e_probe.py --order inproc,cli --skip pread --cli-runs 1 > $O/inproc_first.jsonl 2> $O/inproc_first.err &&
LBF_COPY_THREADS=16 $T 300 python -u tools/c3_e2e_probe.py --order cli,inproc --skip pread > $O/cli_first_t16.jsonl 2> $O/cli_first_t16.err || exit 1
# staging copy helpers kept per worker (CopyPool) vs started per piece, and the
# pinned-ring piece size: pageable host memory in, then 16 files in-process
for k in 1 2; do
  for cfg in "LBF_COPY_POOL=0" "LBF_COPY_POOL=1" "LBF_COPY_POOL=0 LBF_PIN_MB=512"; do
    tag=$(echo $cfg | tr ' =' '__')
    env $cfg $T 120 python -u tools/e2e_sizes.py > $O/e2e_${tag}_$k.json 2> $O/e2e_${tag}_$k.err || exit 1
  done
done
for k in 1 2; do
  for pool in 0 1; do
    LBF_COPY_POOL=$pool $T 200 python -u tools/c3_e2e_probe.py --files 16 --order inproc --skip cli,pread > $O/files16_pool${pool}_$k.jsonl 2> $O/files16_pool${pool}_$k.err || exit 1
  done
done
LBF_COPY_THREADS=8 $T 120 python -u tools/fuzz_host_paths.py --seconds 60 --seed 901 > $O/fuzz_host_paths_pool.txt 2>&1
