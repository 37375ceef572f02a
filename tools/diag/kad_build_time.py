"""Time the Kademlia snapshot table build (ovs_kad_load: k_kad_siblings + k_kad_buckets) at config E's
size (2^24 nodes) -- VERDICT r04 item 7 (182 ms for k_kad_buckets) -- and, with --top-levels, the
sharded build with replicated top buckets.  Prints one JSON line per repetition; a checksum of the
exported tables of a smaller network (--check-nodes) lets two builds be compared for identical
content.

usage: python tools/diag/kad_build_time.py [--nodes 16777216] [--reps 3] [--check-nodes 65536]"""
import argparse
import hashlib
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch

from oversim_amd import KbrEngine, Params, workload as W

ap = argparse.ArgumentParser()
ap.add_argument("--nodes", type=int, default=1 << 24)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--check-nodes", type=int, default=1 << 16)
a = ap.parse_args()
dev = torch.device("cuda", 0)
ids_t, xy_t = W.device_population(a.nodes, 0xC, dev)
torch.cuda.synchronize()
with KbrEngine(0) as e:
    e.set_params(Params.kademlia())
    for r in range(a.reps):
        t = time.perf_counter()
        e.kad_load_device(ids_t.data_ptr(), xy_t.data_ptr(), a.nodes)
        torch.cuda.synchronize()
        print(json.dumps(dict(rep=r, nodes=a.nodes, build_ms=round((time.perf_counter() - t) * 1e3, 2))), flush=True)
net = W.population(a.check_nodes, 0x4B)
with KbrEngine(0) as e:
    e.set_params(Params.kademlia())
    e.kad_load(net.ids, net.xy)
    sib, cnt, nodes = e.kad_tables()
h = hashlib.sha256()
for x in (sib, cnt, nodes):
    h.update(np.ascontiguousarray(x).tobytes())
print(json.dumps(dict(check_nodes=a.check_nodes, tables_sha256=h.hexdigest()[:32])), flush=True)
