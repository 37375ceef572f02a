#!/bin/bash
# Alternative engine library with one object rebuilt from a source under extra flags -- for the
# per-variant objects (e.g. K2's kad_route_a1 = kad_route.hip -DOVS_KAD_A=1 -DOVS_KAD_EX=0).  A/B
# runs load it through OVS_LIB.  usage: tools/build_alt_obj.sh <tag> <source.hip> <object stem> <flags...>
set -e
TAG=$1; SRC=$2; STEM=$3; shift 3
cd "$(dirname "$0")/.."
D=build/alt_$TAG; mkdir -p $D
FL="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off"
/opt/rocm/bin/hipcc $FL "$@" -x hip -c oversim_amd/csrc/$SRC -o $D/$STEM.o
objs=""
for o in build/obj/*.o; do
  b=$(basename $o)
  if [ -f $D/$b ]; then objs="$objs $D/$b"; else objs="$objs $o"; fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o oversim_amd/libovs_kbr_$TAG.so $objs
echo oversim_amd/libovs_kbr_$TAG.so
