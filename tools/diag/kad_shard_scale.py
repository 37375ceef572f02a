"""Diagnose sharded Kademlia at scale on one GPU (world 1): the W = 1 local emulation (no
collectives) and the RCCL path, on workload E populations of a given size."""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch

from oversim_amd import Params, workload as W
from oversim_amd.shard import KadShardStepper, route_kad_local_shards, route_kad_sharded, TorchExchange, done_to_numpy

ap = argparse.ArgumentParser()
ap.add_argument("--nodes", type=int, required=True)
ap.add_argument("--lookups", type=int, required=True)
ap.add_argument("--mode", choices=["local", "nccl"], required=True)
a = ap.parse_args()
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
I = W.bench_inputs("E", dev, world=1, rank=0, seed=1, nodes=a.nodes, n_lookups=a.lookups, sharded=True)
ids = I["ids"] if I["ids"] is not None else I["ids_t"].cpu().numpy().view(np.uint32)
xy = I["xy"] if I["xy"] is not None else I["xy_t"].cpu().numpy()
keys_t, src_t = I["keys_t"], I["src_t"]
torch.cuda.synchronize()
print("population", ids.shape, ids.dtype, xy.shape, keys_t.shape, keys_t.dtype, src_t.dtype,
      int(src_t.max().item()), flush=True)
n = ids.shape[0]
st = KadShardStepper(ids, xy, [0, n], 0, dev, params=Params.kademlia().replace(lookupParallelRpcs=3))
t0 = time.time()
if a.mode == "local":
    done, rounds = route_kad_local_shards([st], [keys_t], [src_t], [0], max_rounds=3000)
    done = done[0]
else:
    import torch.distributed as dist
    dist.init_process_group("nccl", device_id=dev)
    ex = TorchExchange(1, dev)
    done, rounds = route_kad_sharded(st, ex, keys_t, src_t, 0, max_rounds=3000)
torch.cuda.synchronize()
d = done_to_numpy(done)
print(a.mode, "rounds", rounds, "done", len(d), "ok", int((d["status"] == 0).sum()), "hops", float(d["hops"].mean()),
      "s", round(time.time() - t0, 2), flush=True)
if a.mode == "nccl":
    dist.destroy_process_group()
