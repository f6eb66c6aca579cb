#!/bin/bash
# Round-3 GPU session 26: instruction-cache counters of pc4 (7) against
# pc4x2's one-group form (13) at C2 (SQ_WAIT_INST_ANY was 3x higher in 13 with
# the same instruction counts, session 25).
set -o pipefail
O=gpurun_out/r03/s26
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
REPO=${GRAFT_REPO_ROOT:-/root/repo}
export LBF_LIB=$REPO/bitflood_amd/lib/experimental/liblbfhash.so
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE \
  -d $REPO/$O/pmc_ic -o pmc --output-format csv \
  -- python3 $REPO/tools/sweep_variants.py --variants 7,13,12 --max-gib 8 --reps 3 --points 262144:16384,262144:32768 > $REPO/$O/pmc_ic.log 2>&1
