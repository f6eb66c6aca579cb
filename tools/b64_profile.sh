#!/bin/bash
# tools/b64_profile.sh <tag> [lib] -- rocprofv3 evidence for the wire-form kernels
# (b64_decode_canon_kernel, b64_decode_kernel, b64_encode_kernel) on the GPU box,
# driven by tools/b64_rate.py (1,024 x 256 KiB per launch).  [lib] = the
# liblbfhash.so to load (LBF_LIB; default the shipped one), e.g.
# bitflood_amd/lib/ab_r04/liblbfhash.so for round 4's kernels.
#   1. kernel trace + stats (per-kernel durations)
#   2. PMC passes, each in its own run: SQ wave-cycle split and instruction
#      counts; FETCH_SIZE; WRITE_SIZE; LDS and VALU counters; then the TA/TD
#      busy counters (names probed; a pass whose counters this rocprofv3 does not
#      know ends with an ordinary error and is skipped, anything else stops the script)
# Output: gpurun_out/prof/<tag>/...
set -u
TAG=${1:-b64}
LIB=${2:-}
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/prof/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -n "$LIB" ]; then export LBF_LIB=$REPO/$LIB; fi
RATE="$REPO/tools/b64_rate.py"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o trace --output-format csv \
  -- python3 "$RATE" --reps 5 > "$OUT/trace.log" 2>&1 || { echo "trace failed rc=$?"; tail -20 "$OUT/trace.log"; exit 1; }
pass() {  # pass <name> <counters...>
  local name=$1; shift
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc "$@" -d "$OUT/$name" -o pmc --output-format csv \
    -- python3 "$RATE" --reps 1 > "$OUT/$name.log" 2>&1
  local rc=$?
  if [ $rc -eq 0 ]; then echo "pass $name ok"; return 0; fi
  if [ $rc -eq 1 ] || [ $rc -eq 2 ]; then echo "pass $name: rc=$rc (counters not collected)"; tail -3 "$OUT/$name.log"; return 0; fi
  echo "pass $name stopped rc=$rc"; tail -20 "$OUT/$name.log"; exit 1
}
pass pmc_sq SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD \
  SQ_INSTS_VMEM_WR SQ_INSTS_LDS GRBM_GUI_ACTIVE
pass pmc_fetch FETCH_SIZE
pass pmc_write WRITE_SIZE
pass pmc_lds SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_VMEM SQ_BUSY_CYCLES \
  SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE
pass pmc_ta TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TD_TD_BUSY_sum TD_TC_STALL_sum
pass pmc_tcp TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_PENDING_STALL_CYCLES_sum
echo "b64 profile $TAG done"
