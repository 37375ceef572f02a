#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r02z
export OVS_SKIP_BUILD=1
for v in main nodone nostore noxy; do
  if [ $v = main ]; then unset OVS_LIB; else export OVS_LIB=oversim_amd/libovs_kbr_$v.so; fi
  timeout -k 10 120 python tools/diag/chord_shard_speed.py > gpurun_out/r02z/$v.log 2>&1; rc=$?
  echo "$v $rc"; grep -E "step ms|context ms" gpurun_out/r02z/$v.log | tail -n 3
  case $rc in 0) ;; *) exit $rc;; esac
done
