# A/B of library builds through bench.py: tools/ab_bench.sh <out> "<bench args>" <lib.so|current>...
# Three alternating rounds; each line is one bench JSON (parity checked against the goldens).
set -e
out=gpurun_out/$1; args=$2; shift 2
mkdir -p $out
for i in 1 2 3; do
  for lib in "$@"; do
    tag=$(basename $lib .so)
    if [ "$lib" = current ]; then env=""; else env="LBF_LIB=$PWD/$lib"; fi
    env $env timeout -k 10 200 python -u bench.py $args --no-cpu-baseline --no-e2e --no-other-configs > $out/${tag}_$i.json 2> $out/${tag}_$i.err
  done
done
