#!/bin/bash
# Alternative engine library with extra flags on one translation unit (A/B runs through OVS_LIB).
# usage: tools/build_alt_src.sh <tag> <source.hip> <extra hipcc flags...>
set -e
TAG=$1; SRC=$2; shift 2
cd "$(dirname "$0")/.."
D=build/alt_$TAG; mkdir -p $D
FL="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off"
/opt/rocm/bin/hipcc $FL "$@" -x hip -c oversim_amd/csrc/$SRC -o $D/${SRC%.*}.o
objs=""
for o in build/obj/*.o; do
  b=$(basename $o)
  if [ -f $D/$b ]; then objs="$objs $D/$b"; else objs="$objs $o"; fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o oversim_amd/libovs_kbr_$TAG.so $objs
echo oversim_amd/libovs_kbr_$TAG.so
