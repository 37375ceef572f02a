#!/bin/bash
# world-1 rehearsal of the sharded bench paths (RCCL/gloo), small sizes first
set -o pipefail
mkdir -p gpurun_out/r02u
export OVS_SKIP_BUILD=1 OVS_BENCH_SHARD=1
p=29620
for be in gloo nccl; do
  p=$((p+1))
  OVS_BENCH_BACKEND=$be timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
    --master-addr 127.0.0.1 --master-port $p bench.py --gpus 1 --workload E --nodes 65536 --lookups 20000 \
    --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/r02u/E_$be.json 2> gpurun_out/r02u/E_$be.err
  echo "E $be exit $?"; tail -2 gpurun_out/r02u/E_$be.json gpurun_out/r02u/E_$be.err
done
p=$((p+1))
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port $p bench.py --gpus 1 --workload C --steps 5 --warmup 2 --no-cpu-baseline \
  > gpurun_out/r02u/C_nccl.json 2> gpurun_out/r02u/C_nccl.err
echo "C exit $?"; tail -2 gpurun_out/r02u/C_nccl.json gpurun_out/r02u/C_nccl.err
