#!/bin/bash
# Round-3 GPU session 8: where C3's end-to-end EncodeFile time goes
# (tools/c3_e2e_probe.py: cold CLI, warm in-process batch, host pread alone),
# then the session-7 fuzz pass over the round's host-side changes.
set -o pipefail
O=gpurun_out/r03/s8
mkdir -p $O
T="timeout -k 10"
$T 400 python -u tools/c3_e2e_probe.py > $O/c3_e2e_probe.jsonl 2> $O/c3_e2e_probe.err &&
bash tools/r03_session7.sh
