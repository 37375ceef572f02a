#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r02w
export OVS_SKIP_BUILD=1 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29651
timeout -k 10 150 python tools/diag/kad_shard_scale.py --nodes 16777216 --lookups 1000000 --mode local > gpurun_out/r02w/a.log 2>&1; rc=$?; echo "a $rc"; tail -n 3 gpurun_out/r02w/a.log; case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 150 python tools/diag/kad_shard_scale.py --nodes 4194304 --lookups 4000000 --mode local > gpurun_out/r02w/b.log 2>&1; rc=$?; echo "b $rc"; tail -n 3 gpurun_out/r02w/b.log; case $rc in 124|134|137|139) exit $rc;; esac
export MASTER_PORT=29652
timeout -k 10 150 python tools/diag/kad_shard_scale.py --nodes 4194304 --lookups 4000000 --mode nccl > gpurun_out/r02w/c.log 2>&1; rc=$?; echo "c $rc"; tail -n 3 gpurun_out/r02w/c.log; case $rc in 124|134|137|139) exit $rc;; esac
