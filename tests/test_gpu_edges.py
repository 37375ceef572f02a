"""Edge inputs through the C ABI on every routed overlay: empty batches return at once with nothing
written, and a host-pointer batch whose source lies outside the network is refused with
OVS_EINVAL before any kernel reads it (ovs_kbr.h: ovs_route_batch / ovs_lookup_batch)."""
from __future__ import annotations

import numpy as np
import pytest

from oversim_amd import KbrEngine, KbrError, Params, workload as W

pytestmark = pytest.mark.gpu


def _load(engine: KbrEngine, overlay: str, n: int = 500):
    net = W.population(n, 31)
    if overlay == "chord":
        engine.set_params(Params.chord())
        engine.chord_load(net.ids, net.xy)
    elif overlay == "kademlia":
        engine.set_params(Params.kademlia())
        engine.kad_load(net.ids, net.xy)
    else:
        engine.set_params(Params.koorde())
        engine.koorde_load(net.ids, net.xy)
    return net


@pytest.mark.parametrize("overlay", ["chord", "kademlia", "koorde"])
def test_empty_batch(engine: KbrEngine, overlay):
    _load(engine, overlay)
    r = engine.lookup(np.zeros((0, 5), np.uint32), np.zeros(0, np.uint32), record_hops=True)
    assert all(len(v) == 0 for v in r.values())
    if overlay != "koorde":
        c = engine.lookupCall(np.zeros((0, 5), np.uint32), np.zeros(0, np.uint32))
        assert all(len(v) == 0 for v in c.values())


@pytest.mark.parametrize("overlay", ["chord", "kademlia", "koorde"])
def test_source_outside_the_network_is_refused(engine: KbrEngine, overlay):
    net = _load(engine, overlay)
    rng = np.random.default_rng(5)
    keys = W.random_keys(100, rng)
    src = rng.integers(0, len(net.ids), 100).astype(np.uint32)
    ok = engine.lookup(keys, src)                        # the valid batch routes
    for bad in (len(net.ids), 0xFFFFFFFF):
        s2 = src.copy()
        s2[57] = bad
        with pytest.raises(KbrError, match="source index out of range"):
            engine.lookup(keys, s2)
        if overlay != "koorde":
            with pytest.raises(KbrError, match="source index out of range"):
                engine.lookupCall(keys, s2)
    again = engine.lookup(keys, src)                     # the context is still usable, results unchanged
    for f in ok:
        assert np.array_equal(ok[f], again[f]), f
