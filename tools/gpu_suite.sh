#!/bin/bash
# tools/gpu_suite.sh <tag> -- one GPU-box pass: the -m gpu suite, the
# Base64Encode latency probe, the C2 bench and a 2-rank bench rehearsal
# (two ranks on the one GPU, gloo), each step under its own time limit and
# stopping at the first step that fails.  Logs land in gpurun_out/<tag>/.
set -o pipefail
tag=${1:-run}
only=${2:-}  # optional pytest -k expression
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=${TMPDIR:-/tmp}
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$secs" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 5 "$out/$name.log"
  return $rc
}
step pytest_gpu 700 python -u -m pytest tests -m gpu -v -rP --durations=15 --timeout 300 --timeout-method thread -p no:cacheprovider ${only:+-k "$only"} &&
step latency 120 bitflood_amd/lib/lbf_latency --reps 200 &&
step bench_c2 300 python bench.py --steps 20 --warmup 5 &&
step bench_2rank_gloo 300 env LBF_BENCH_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2
