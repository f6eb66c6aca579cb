#!/bin/bash
# Round-3 GPU session 25: SQ counters of pc4 (7) against pc4x2's one-group form
# (13) at C2 -- where do 13's extra cycles go (LDS bank conflicts, instruction
# fetch, issue waits)?  Counter passes only (--pmc with --kernel-trace).
set -o pipefail
O=gpurun_out/r03/s25
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
REPO=${GRAFT_REPO_ROOT:-/root/repo}
export LBF_LIB=$REPO/bitflood_amd/lib/experimental/liblbfhash.so
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_IFETCH SQ_WAIT_INST_LDS -d $REPO/$O/pmc_a -o pmc --output-format csv \
  -- python3 $REPO/tools/sweep_variants.py --variants 7,13 --max-gib 4 --reps 3 --points 262144:16384 > $REPO/$O/pmc_a.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU \
  SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $REPO/$O/pmc_b -o pmc --output-format csv \
  -- python3 $REPO/tools/sweep_variants.py --variants 7,13 --max-gib 4 --reps 3 --points 262144:16384 > $REPO/$O/pmc_b.log 2>&1
