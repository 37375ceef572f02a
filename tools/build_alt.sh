#!/bin/bash
# Build an alternative engine library with extra flags on the K2 route objects only, for A/B
# runs (OVS_LIB=oversim_amd/libovs_kbr_<tag>.so python bench.py ...).  The main build must be
# current (python -m oversim_amd.build).
# usage: tools/build_alt.sh <tag> <extra hipcc flags...>
set -e
TAG=$1; shift
cd "$(dirname "$0")/.."
D=build/alt_$TAG; mkdir -p $D
FL="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off"
pids=()
for a in 1 2 3 4; do for x in 0 1; do
  s=""; [ $x = 1 ] && s=x
  /opt/rocm/bin/hipcc $FL -DOVS_KAD_A=$a -DOVS_KAD_EX=$x "$@" -x hip -c oversim_amd/csrc/kad_route.hip -o $D/kad_route_a$a$s.o 2>/dev/null &
  pids+=($!)
done; done
for p in "${pids[@]}"; do wait $p; done
objs=""
for o in build/obj/*.o; do
  b=$(basename $o)
  if [ -f $D/$b ]; then objs="$objs $D/$b"; else objs="$objs $o"; fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o oversim_amd/libovs_kbr_$TAG.so $objs
echo oversim_amd/libovs_kbr_$TAG.so
