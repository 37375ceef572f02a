#!/bin/bash
# world-1 sharded bench paths without torchrun: C under the kernel trace, E at growing sizes
set -o pipefail
mkdir -p gpurun_out/r02v
export OVS_SKIP_BUILD=1 OVS_BENCH_SHARD=1 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1
export MASTER_PORT=29641
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r02v/profC -o run -- python bench.py --gpus 1 --workload C \
  --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r02v/C.json 2> gpurun_out/r02v/C.err || exit 1
echo "C done"
export MASTER_PORT=29642
timeout -k 10 200 python bench.py --gpus 1 --workload E --nodes 4194304 --lookups 1000000 --steps 1 --warmup 0 \
  --no-cpu-baseline > gpurun_out/r02v/E22.json 2> gpurun_out/r02v/E22.err || exit 2
echo "E22 done"
export MASTER_PORT=29643
timeout -k 10 240 python bench.py --gpus 1 --workload E --steps 1 --warmup 0 \
  --no-cpu-baseline > gpurun_out/r02v/E24.json 2> gpurun_out/r02v/E24.err || exit 3
echo "E24 done"
