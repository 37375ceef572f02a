#!/bin/bash
# Build an alternative engine library with extra flags on the K2 route objects only, for A/B
# runs (OVS_LIB=oversim_amd/libovs_kbr_<tag>.so python bench.py ...).  The main build must be
# current (python -m oversim_amd.build).  OVS_ALT_OBJS (default "a1 a3": the non-exact alpha = 1
# and 3 objects that bench workloads B, E and R run) selects which K2 objects are rebuilt; the
# others are the main build's.
# usage: tools/build_alt.sh <tag> <extra hipcc flags...>
set -e
TAG=$1; shift
cd "$(dirname "$0")/.."
D=build/alt_$TAG; mkdir -p $D
FL="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off"
pids=()
for o in ${OVS_ALT_OBJS:-a1 a3}; do
  a=${o:1:1}; x=0; [ "${o:2:1}" = x ] && x=1
  /opt/rocm/bin/hipcc $FL -DOVS_KAD_A=$a -DOVS_KAD_EX=$x "$@" -x hip -c oversim_amd/csrc/kad_route.hip -o $D/kad_route_$o.o 2>/dev/null &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
objs=""
for o in build/obj/*.o; do
  b=$(basename $o)
  if [ -f $D/$b ]; then objs="$objs $D/$b"; else objs="$objs $o"; fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o oversim_amd/libovs_kbr_$TAG.so $objs
echo oversim_amd/libovs_kbr_$TAG.so
