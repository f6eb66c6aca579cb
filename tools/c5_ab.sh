#!/bin/bash
# tools/c5_ab.sh <tag> <rounds> [variants] -- alternating A/B runs of the C5 transfer
# (16 GiB at 256 KiB, window 4096, batch <= 1024, every 1000th chunk corrupted
# once, generated seeder) on the GPU box, one JSON line per run appended to
# gpurun_out/<tag>/c5_ab.jsonl with the variant's name.  Variants (lbf_loopback
# flags): r03 = one verifier, serial seeder (round 3's pipeline); v1 = one
# verifier, pipelined seeder; v2 = two verifiers, pipelined seeder; v2s = two
# verifiers, serial seeder; gd = v2s with the leecher's base64 decode on the
# GPU (the default since round 4); gd1 = gd with one verifier; ge = gd with
# the seeder's base64 encode on the GPU too (--gpu-encode); sw2 = gd with two
# seeder workers; sw2e = sw2 with --gpu-encode; sw3 = gd with three seeder workers;
# gd3 / gd4 = gd with three / four leecher verifiers;
# pre = v2s run by bitflood_amd/lib/lbf_loopback_prepool when that binary exists
# (a build of an earlier lbf_loopback.cpp, for an A/B across a harness change);
# 1p / 2p = the defaults as one process (--role both) / as the reference's two
# processes, a seeder process and a leecher process (tests/c5_pair.py).
set -o pipefail
tag=${1:-c5ab}
rounds=${2:-2}
variants=${3:-"r03 v2 v1 v2s"}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=${TMPDIR:-/tmp}
declare -A flags=([r03]="--verifiers 1 --cpu-decode" [v1]="--verifiers 1 --pipelined-seeder --cpu-decode" \
                  [v2]="--verifiers 2 --pipelined-seeder --cpu-decode" [v2s]="--verifiers 2 --cpu-decode" \
                  [gd]="--verifiers 2 --gpu-decode" [gd1]="--verifiers 1 --gpu-decode" \
                  [ge]="--verifiers 2 --gpu-decode --gpu-encode" \
                  [sw2]="--verifiers 2 --seeder-workers 2" [sw2e]="--verifiers 2 --seeder-workers 2 --gpu-encode" \
                  [sw3]="--verifiers 2 --seeder-workers 3" \
                  [gd3]="--verifiers 3" [gd4]="--verifiers 4" [pre]="--verifiers 2" [1p]="" [2p]="")
for r in $(seq "$rounds"); do
  for v in $variants; do
    bin=bitflood_amd/lib/lbf_loopback
    if [ "$v" = pre ]; then bin=bitflood_amd/lib/lbf_loopback_prepool; fi
    run=$bin
    if [ "$v" = 2p ]; then run="python3 -m tests.c5_pair"; fi
    line=$(timeout -k 10 240 $run --size $((16 << 30)) --chunksize 262144 --window 4096 \
      --batch 1024 --corrupt 1000 --synthetic --threads 16 $([ "$v" = 2p ] || echo --dir "$TMPDIR/c5ab") ${flags[$v]} 2> "$out/$v.$r.err") \
      || { echo "run $v.$r failed rc=$?"; tail -5 "$out/$v.$r.err"; exit 1; }
    echo "{\"variant\": \"$v\", \"round\": $r, \"run\": $line}" >> "$out/c5_ab.jsonl"
    echo "$v.$r done"
  done
done
