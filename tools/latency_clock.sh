# Effective clock of the single-chunk Base64Encode latency path (one chain on
# one CU): kernel trace + GRBM_GUI_ACTIVE in one PMC pass over lbf_latency.
set -o pipefail
out=$PWD/gpurun_out/latclk
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES -d $out/pmc -o pmc --output-format csv \
  -- $GRAFT_REPO_ROOT/bitflood_amd/lib/lbf_latency --reps 50 > $out/pmc.log 2>&1
