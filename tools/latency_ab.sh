# tools/latency_ab.sh <out> <lib.so|current>... : tools/latency_ab.py per build, twice
set -e
out=gpurun_out/$1; shift
mkdir -p $out
for i in 1 2; do
  for lib in "$@"; do
    tag=$(basename $lib .so)
    if [ "$lib" = current ]; then env=""; else env="LBF_LIB=$PWD/$lib"; fi
    env $env timeout -k 10 120 python -u tools/latency_ab.py 50 > $out/${tag}_$i.json 2> $out/${tag}_$i.err
  done
done
