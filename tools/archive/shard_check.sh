#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r02s
export OVS_SKIP_BUILD=1 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29671
chk() { case $1 in 0) ;; *) exit $1;; esac; }
timeout -k 10 150 python tools/diag/chord_shard_speed.py > gpurun_out/r02s/chord.log 2>&1; rc=$?; echo "chord $rc"; tail -n 9 gpurun_out/r02s/chord.log; chk $rc
timeout -k 10 150 python tools/diag/kad_shard_scale.py --nodes 4194304 --lookups 4000000 --mode nccl > gpurun_out/r02s/kad.log 2>&1; rc=$?; echo "kad $rc"; tail -n 2 gpurun_out/r02s/kad.log; chk $rc
timeout -k 10 400 python -u -m pytest tests/test_shard.py -x -v --timeout 200 --timeout-method thread -m gpu > gpurun_out/r02s/tests.log 2>&1; rc=$?; echo "tests $rc"; tail -n 5 gpurun_out/r02s/tests.log; chk $rc
