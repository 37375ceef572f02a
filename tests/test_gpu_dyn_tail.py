"""The persistent route kernels' dynamic tail: a batch's last 30 % is handed out from
a per-launch device counter taken from the context's slot pool.  Concurrent device-pointer calls on
different streams of one context, and more calls than the pool has slots, must each see their own
counter: every result equals the same batch routed alone with static slices (OVS_NO_DYN=1)."""
from __future__ import annotations

import os

import numpy as np
import pytest

from oversim_amd import KbrEngine, Params, workload as W

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("overlay", ["chord", "kademlia"])
def test_concurrent_streams_share_no_counter(engine: KbrEngine, overlay, monkeypatch):
    import torch
    dev = torch.device("cuda", 0)
    net = W.population(1 << 16, 91)
    if overlay == "chord":
        engine.set_params(Params.chord())
        engine.chord_load(net.ids, net.xy)
    else:
        engine.set_params(Params.kademlia().replace(lookupParallelRpcs=3))
        engine.kad_load(net.ids, net.xy)
    n = 1 << 18                                       # the dynamic tail's threshold
    batches = []
    for b in range(3):
        keys, src = W.lookups(net.ids, n, 100 + b, node_ids=False)
        batches.append((torch.from_numpy(keys.view(np.int32)).to(dev), torch.from_numpy(src.view(np.int32)).to(dev)))
    # reference: each batch alone, static slices
    monkeypatch.setenv("OVS_NO_DYN", "1")
    ref = []
    for k, s in batches:
        o = torch.empty((n, 16), dtype=torch.uint8, device=dev)
        engine.lookup_device(k.data_ptr(), s.data_ptr(), n, o.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        ref.append(o.cpu().numpy())
    monkeypatch.delenv("OVS_NO_DYN")
    # 40 launches (more than the 32 slots) over three streams, queued without waiting
    streams = [torch.cuda.Stream(device=dev) for _ in range(3)]
    outs = []
    for i in range(40):
        b = i % 3
        k, s = batches[b]
        o = torch.empty((n, 16), dtype=torch.uint8, device=dev)
        engine.lookup_device(k.data_ptr(), s.data_ptr(), n, o.data_ptr(), streams[b].cuda_stream)
        outs.append((b, o))
    torch.cuda.synchronize()
    for i, (b, o) in enumerate(outs):
        assert np.array_equal(o.cpu().numpy(), ref[b]), f"launch {i} (batch {b}) differs from the static route"
