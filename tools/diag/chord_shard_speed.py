"""Time the Chord shard-step kernel (W = 1, one cohort, no collectives) against the unsharded
route kernel on the same ring and lookups (workload C inputs)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch

from oversim_amd import KbrEngine, Params, workload as W
from oversim_amd.shard import GpuShardStepper, route_local_shards, done_to_numpy

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
m = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
I = W.bench_inputs("C", dev, world=1, rank=0, seed=1, n_lookups=m, sharded=True)
ids = I["ids"] if I["ids"] is not None else I["ids_t"].cpu().numpy().view(np.uint32)
xy = I["xy"] if I["xy"] is not None else I["xy_t"].cpu().numpy()
keys_t, src_t = I["keys_t"], I["src_t"]
n = ids.shape[0]
torch.cuda.synchronize()

eng = KbrEngine(0)
eng.set_params(Params.chord())
eng.chord_load_device(I["ids_t"].data_ptr(), I["xy_t"].data_ptr(), n)
dout = torch.empty((m, 16), dtype=torch.uint8, device=dev)
for rep in range(3):
    torch.cuda.synchronize(); t0 = time.time()
    eng.lookup_device(keys_t.data_ptr(), src_t.data_ptr(), m, dout.data_ptr())
    torch.cuda.synchronize(); print("unsharded ms", round((time.time() - t0) * 1e3, 2), flush=True)

st = GpuShardStepper(ids, xy, [0, n], 0, dev, capacity=m + m // 4)
for rep in range(3):
    st.reset(m + 1024)
    inbox = st.make_records(keys_t, src_t, 0)
    torch.cuda.synchronize(); t0 = time.time()
    out, cnt = st.step(inbox)
    torch.cuda.synchronize(); t1 = time.time()
    print("shard step ms", round((t1 - t0) * 1e3, 2), "sent", cnt.tolist(), "done", int(st.done_count.item()), flush=True)
for rep in range(2):
    torch.cuda.synchronize(); t0 = time.time()
    st.eng.lookup_device(keys_t.data_ptr(), src_t.data_ptr(), m, dout.data_ptr())
    torch.cuda.synchronize(); print("unsharded kernel on the shard context ms", round((time.time() - t0) * 1e3, 2), flush=True)
import ctypes as C
from oversim_amd.kbr import lib
for rep in range(2):
    st.reset(m + 1024)
    inbox = st.make_records(keys_t, src_t, 0)
    torch.cuda.synchronize(); t0 = time.time()
    r = lib().ovs_shard_step(eng._h, C.c_void_p(inbox.data_ptr()), m, C.c_void_p(st._out[0].data_ptr()), st._cap[0],
                             C.c_void_p(st._cnt[0].data_ptr()), C.c_void_p(st.done.data_ptr()), st.done_cap,
                             C.c_void_p(st.done_count.data_ptr()), st._lo, 1, C.c_void_p(0))
    torch.cuda.synchronize(); print("shard kernel on the unsharded context ms", r, round((time.time() - t0) * 1e3, 2), flush=True)
d = done_to_numpy(st.finished())
print("shard hops mean", float(d["hops"].mean()), "ok", int((d["status"] == 0).sum()))
