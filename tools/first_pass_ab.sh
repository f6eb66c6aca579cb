# A/B of the first job on a fresh context: tools/first_pass_ab.sh <out> <lib.so|current>...
set -e
out=gpurun_out/$1; shift
mkdir -p $out
for i in 1 2; do
  for lib in "$@"; do
    tag=$(basename $lib .so)
    if [ "$lib" = current ]; then env=""; else env="LBF_LIB=$PWD/$lib"; fi
    env $env timeout -k 10 240 python -u tools/first_pass.py 3 > $out/${tag}_$i.log 2>&1
  done
done
