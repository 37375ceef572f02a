"""K1 batch-order A/B: config C's 10M random-key lookups routed by K1 in the
caller's (random) order, bucketed by the top B bits of the key (the order a counting sort on those
bits would give, bucket order inside unchanged), and fully sorted.  Kernel time per launch with HIP
events; the order is prepared on the host, outside the timing -- this is the upper bound of what an
in-step counting sort could gain before paying for itself.

usage: python tools/diag/k1_locality_ab.py [--bits 10 12 14 16] [--reps 10]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch

from oversim_amd import KbrEngine, Params, workload as W

ap = argparse.ArgumentParser()
ap.add_argument("--bits", type=int, nargs="*", default=[8, 10, 12, 14, 16])
ap.add_argument("--reps", type=int, default=10)
a = ap.parse_args()
dev = torch.device("cuda", 0)
I = W.bench_inputs("C", dev)
n, m = I["n_total"], I["m"]
keys = I["keys_t"].cpu().numpy().view(np.uint32).reshape(m, 5)
src = I["src_t"].cpu().numpy().view(np.uint32)
eng = KbrEngine(0)
eng.set_params(Params.chord())
torch.cuda.synchronize()
eng.chord_load_device(I["ids_t"].data_ptr(), I["xy_t"].data_ptr(), n)
stream = torch.cuda.Stream(device=dev)


def run(order, label):
    k = torch.from_numpy(np.ascontiguousarray(keys[order]).view(np.int32)).to(dev)
    s = torch.from_numpy(np.ascontiguousarray(src[order]).view(np.int32)).to(dev)
    out = torch.empty((m, 16), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    for _ in range(2):
        eng.lookup_device(k.data_ptr(), s.data_ptr(), m, out.data_ptr(), stream.cuda_stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(a.reps):
        eng.lookup_device(k.data_ptr(), s.data_ptr(), m, out.data_ptr(), stream.cuda_stream)
    e1.record(stream)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.reps
    o = out.cpu().numpy().reshape(-1, 16)
    hops = int(o[:, 4:6].copy().view(np.uint16).astype(np.int64).sum())
    print(json.dumps({"order": label, "kernel_ms": round(ms, 4), "hops": hops}), flush=True)
    return o


base = run(np.arange(m), "random (caller order)")
top = keys[:, 4].astype(np.uint64)
for b in a.bits:
    order = np.argsort(top >> np.uint64(32 - b), kind="stable")
    o = run(order, f"bucketed top {b} bits")
    inv = np.empty(m, dtype=np.int64)
    inv[order] = np.arange(m)
    assert np.array_equal(o[inv], base), "results differ from the caller-order route"
full = np.lexsort(tuple(keys[:, i] for i in range(5)))
o = run(full, "fully sorted")
