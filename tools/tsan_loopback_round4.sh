#!/bin/bash
# tools/tsan_loopback_round4.sh -- ThreadSanitizer over the C5 harness with the round-4 options
# (seeder workers, GPU encode, pipelined seeder with three verifiers); run on the GPU box.
set -o pipefail
mkdir -p gpurun_out/tsan2 /tmp/ts
timeout -k 10 500 bash tools/tsan_build.sh > gpurun_out/tsan2/build.txt 2>&1 || exit 1
export TSAN_OPTIONS="halt_on_error=1 report_signal_unsafe=0 suppressions=tools/tsan.supp"
for args in "--verifiers 2 --seeder-workers 2" "--verifiers 2 --seeder-workers 2 --gpu-encode" "--verifiers 3 --seeder-workers 3 --pipelined-seeder --cpu-decode"; do
  timeout -k 10 240 tools/build/tsan/tsan_loopback --size $((256 << 20)) --chunksize 65536 --window 512 --batch 128 --corrupt 7 --synthetic --threads 8 --dir /tmp/ts $args > gpurun_out/tsan2/run.json 2> gpurun_out/tsan2/run.err || { echo "tsan run failed: $args rc=$?"; tail -40 gpurun_out/tsan2/run.err; exit 1; }
  echo "{\"args\": \"$args\", \"run\": $(cat gpurun_out/tsan2/run.json)}" >> gpurun_out/tsan2/tsan_loopback.jsonl
  echo "ok: $args"
done
