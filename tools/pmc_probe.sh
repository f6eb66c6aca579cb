#!/bin/bash
# tools/pmc_probe.sh -- SQ/SQC counters on the compute-only SHA-1 probe (diagnostic).
set -u
REPO=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$REPO/gpurun_out/pmcprobe
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
grep -oE "(SQ|SQC)_[A-Z0-9_]+" "$OUT/counters.txt" | sort -u > "$OUT/sq_counters.txt" || true
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" "SQ_INSTS_VALU SQ_IFETCH SQC_ICACHE_MISSES SQC_ICACHE_HITS" "SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VALU GRBM_GUI_ACTIVE"; do
  tag=$(echo $set | cut -d' ' -f1)
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $set -d "$OUT/$tag" -o pmc --output-format csv \
    -- "$REPO/tools/build/probe_placement" 262144 256 0 > "$OUT/$tag.log" 2>&1 || echo "pmc $tag failed rc=$?"
done
echo done
