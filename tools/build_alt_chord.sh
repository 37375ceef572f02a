#!/bin/bash
# Alternative engine library with extra flags on chord.hip only (A/B runs through OVS_LIB).
# usage: tools/build_alt_chord.sh <tag> <extra hipcc flags...>
set -e
TAG=$1; shift
cd "$(dirname "$0")/.."
D=build/alt_$TAG; mkdir -p $D
FL="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off"
/opt/rocm/bin/hipcc $FL "$@" -x hip -c oversim_amd/csrc/chord.hip -o $D/chord.o
objs=""
for o in build/obj/*.o; do
  b=$(basename $o)
  if [ -f $D/$b ]; then objs="$objs $D/$b"; else objs="$objs $o"; fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o oversim_amd/libovs_kbr_$TAG.so $objs
echo oversim_amd/libovs_kbr_$TAG.so
