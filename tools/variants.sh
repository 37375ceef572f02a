#!/bin/bash
# Build experimental variants of libovs_kbr.so with extra -D flags into build/var/<name>/.
# usage: tools/variants.sh name "-DFOO=1 -DBAR=2" [name2 "flags2" ...]
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
while [ $# -gt 0 ]; do
  N=$1; F=$2; shift 2
  D=$ROOT/build/var/$N; mkdir -p $D
  OBJS=""
  for src in chord.hip kad.hip kad_shard.hip stats.hip ovs_kbr.cpp ovs_ini.cpp; do
    o=$D/${src%.*}.o
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -w $F -x hip -c $ROOT/oversim_amd/csrc/$src -o $o &
    OBJS="$OBJS $o"
  done
  wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $D/libovs_kbr.so $OBJS
  echo built $D/libovs_kbr.so
done
