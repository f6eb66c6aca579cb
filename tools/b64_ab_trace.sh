#!/bin/bash
# tools/b64_ab_trace.sh <tag> <rounds> <lib>... -- alternating kernel traces of
# the wire kernels (tools/b64_rate.py, 1,024 x 256 KiB per launch) for A/B
# builds (tools/b64_ab_build.sh); "shipped" = the in-tree library.  Per run:
# gpurun_out/prof/<tag>/<name>.<round>/trace_kernel_stats.csv
set -u
tag=$1; rounds=$2; shift 2
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
for r in $(seq "$rounds"); do
  for lib in "$@"; do
    name=$lib
    if [ "$lib" = shipped ]; then unset LBF_LIB; else export LBF_LIB=$REPO/bitflood_amd/lib/ab_$lib/liblbfhash.so; fi
    out=$REPO/gpurun_out/prof/$tag/$name.$r
    mkdir -p "$out"
    (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$out" -o trace --output-format csv \
      -- python3 "$REPO/tools/b64_rate.py" --reps 5 > "$out/run.log" 2>&1) || { echo "$name.$r failed rc=$?"; tail -5 "$out/run.log"; exit 1; }
    echo "$name.$r done"
  done
done
