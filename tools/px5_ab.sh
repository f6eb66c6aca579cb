# A/B of pcx5 (C4) builds: tools/px5_ab.sh <out-dir> <lib.so|current>...
# Two rounds over the builds, each a C4 bench with parity against the golden.
set -e
out=gpurun_out/$1; shift
mkdir -p $out
for i in 1 2; do
  for lib in "$@"; do
    tag=$(basename $lib .so)
    if [ "$lib" = current ]; then env=""; else env="LBF_LIB=$PWD/$lib"; fi
    env $env timeout -k 10 200 python -u bench.py --config c4 --no-cpu-baseline --no-e2e > $out/${tag}_$i.json 2> $out/${tag}_$i.err
  done
done
