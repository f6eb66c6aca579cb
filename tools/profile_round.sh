#!/bin/bash
# tools/profile_round.sh -- run on the GPU box (via gpurun) to collect the
# rocprofv3 evidence for one bench configuration, all in one lease.
#   0. the plain bench line first, unprofiled (bench.json): the same lease's
#      ms_per_step, which the trace's median must match (tools/pmc_traffic.py)
#   1. kernel trace + stats of bench.py (per-kernel average duration)
#   2. PMC passes (each in its own run): SQ issue/wait counters, FETCH_SIZE, WRITE_SIZE
# Output: $GRAFT_REPO_ROOT/gpurun_out/prof/<tag>/...
# Usage: tools/profile_round.sh <tag> [extra bench args...]   (one rank: no --gpus N>1,
# bench.py refuses to start its own ranks under the profiler)
set -u
TAG=${1:-run}
shift || true
REPO=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$REPO/gpurun_out/prof/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 python3 "$REPO/bench.py" $* > "$OUT/bench.json" 2> "$OUT/bench.err" \
  || { echo "bench run failed rc=$?"; tail -20 "$OUT/bench.err"; exit 1; }
# trace pass: the bench command exactly as the driver runs it (default flags)
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o trace --output-format csv \
  -- python3 "$REPO/bench.py" $* > "$OUT/trace.log" 2>&1 || { echo "trace run failed rc=$?"; tail -20 "$OUT/trace.log"; exit 1; }
# counter passes: same workload, fewer steps, no CPU leg
BENCH="$REPO/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e $*"

timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY \
  SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE \
  -d "$OUT/pmc_sq" -o pmc --output-format csv -- python3 $BENCH > "$OUT/pmc_sq.log" 2>&1 \
  || { echo "pmc_sq failed rc=$?"; tail -20 "$OUT/pmc_sq.log"; exit 1; }

timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o pmc --output-format csv \
  -- python3 $BENCH > "$OUT/pmc_fetch.log" 2>&1 || { echo "pmc_fetch failed rc=$?"; tail -20 "$OUT/pmc_fetch.log"; exit 1; }

timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$OUT/pmc_write" -o pmc --output-format csv \
  -- python3 $BENCH > "$OUT/pmc_write.log" 2>&1 || { echo "pmc_write failed rc=$?"; tail -20 "$OUT/pmc_write.log"; exit 1; }
echo "profile $TAG done"
