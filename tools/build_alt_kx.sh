#!/bin/bash
# Build an alternative engine library with extra flags on K2x (kad_refresh.hip) only, for A/B runs
# (tools/gpu_ab.sh).  The main build must be current.  usage: tools/build_alt_kx.sh <tag> <flags...>
set -e
TAG=$1; shift
cd "$(dirname "$0")/.."
D=build/alt_$TAG; mkdir -p $D
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off "$@" -x hip -c oversim_amd/csrc/kad_refresh.hip -o $D/kad_refresh.o 2>/dev/null
objs=""
for o in build/obj/*.o; do
  b=$(basename $o)
  if [ -f $D/$b ]; then objs="$objs $D/$b"; else objs="$objs $o"; fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o oversim_amd/libovs_kbr_$TAG.so $objs
echo oversim_amd/libovs_kbr_$TAG.so
