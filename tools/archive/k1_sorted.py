"""K1 batch-order experiment: route config C's 10M random-key lookups in their
generated order, pre-sorted by key (sorted outside the timed region: the kernel's own effect), and
sorted inside the timed region (sort by the key's top 32 bits, gather keys/sources, route, scatter
the 16 B results back).  Prints ms per step of each; run under rocprofv3 --pmc FETCH_SIZE with a mode
argument (plain | presorted) to count the lines.  usage: k1_sorted.py [all|plain|presorted] [steps]"""
from __future__ import annotations

import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
from oversim_amd import KbrEngine, Params, workload as W  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "all"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
dev = torch.device("cuda", 0)
I = W.bench_inputs("C", dev, world=1, rank=0)
n, m = I["n_total"], I["m"]
keys, src = I["keys_t"], I["src_t"]
eng = KbrEngine(0)
eng.set_params(Params.chord())
torch.cuda.synchronize()
eng.chord_load_device(I["ids_t"].data_ptr(), I["xy_t"].data_ptr(), n)
stream = torch.cuda.Stream(device=dev)
out = torch.empty((m, 16), dtype=torch.uint8, device=dev)
top = keys[:, 4].to(torch.int64) & 0xFFFFFFFF
perm = torch.sort(top).indices
skeys, ssrc = keys[perm].contiguous(), src[perm].contiguous()
sout = torch.empty_like(out)


def route(k, s, o):
    eng.lookup_device(k.data_ptr(), s.data_ptr(), m, o.data_ptr(), stream.cuda_stream)


def sorted_step():
    p = torch.sort(keys[:, 4].to(torch.int64) & 0xFFFFFFFF).indices
    k2, s2 = keys[p], src[p]
    route(k2, s2, sout)
    out[p] = sout


def timed(fn):
    torch.cuda.set_stream(stream)
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(steps):
        fn()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / steps


res = {"lookups": m, "nodes": n}
if mode in ("all", "plain"):
    res["plain_ms"] = timed(lambda: route(keys, src, out))
    ref = out.clone()
if mode in ("all", "presorted"):
    res["presorted_kernel_ms"] = timed(lambda: route(skeys, ssrc, sout))
if mode == "all":
    res["sorted_in_step_ms"] = timed(sorted_step)
    assert torch.equal(out, ref), "sorted batch: results differ from the generated order's"
    o = ref.cpu().numpy()
    res["hops"] = int(o[:, 4:6].copy().view(np.uint16).astype(np.int64).sum())
print(json.dumps(res), flush=True)
