"""The oracle's lazy networks (tables evaluated per access, used for the D/E samples) give the
same tables and the same lookups as the stored (eager) tables.  CPU only."""
from __future__ import annotations

import numpy as np
import pytest

from oversim_amd import workload as W
from oracle_lib import OracleNet, chord_params, kad_params

FIELDS = ("responsible", "hops", "status", "one_way_hops", "latency_ns")


def _same(a: dict, b: dict, extra=()):
    for f in FIELDS + tuple(extra):
        assert np.array_equal(a[f], b[f]), f


def test_chord_lazy_matches_eager():
    net = W.population(5000, 91)
    e = OracleNet("chord", net.ids, net.xy)
    z = OracleNet("chord", net.ids, net.xy, lazy=True)
    assert np.array_equal(e.chord_fingers(), z.chord_fingers())
    k1, s1 = W.lookups(net.ids, 3000, 92, node_ids=True)
    k2, s2 = W.lookups(net.ids, 3000, 93, node_ids=False)
    keys, src = np.concatenate([k1, k2]), np.concatenate([s1, s2])
    _same(e.route(keys, src), z.route(keys, src), ("hop_seq",))
    p = chord_params(routingType=1)
    _same(OracleNet("chord", net.ids, net.xy, p).route(keys, src),
          OracleNet("chord", net.ids, net.xy, p, lazy=True).route(keys, src), ("hop_seq",))


def test_chord_lazy_fix_fingers_materialises():
    net = W.population(600, 94)
    e = OracleNet("chord", net.ids, net.xy)
    z = OracleNet("chord", net.ids, net.xy, lazy=True)
    assert e.chord_fix_fingers() == z.chord_fix_fingers()
    assert np.array_equal(e.chord_fingers(), z.chord_fingers())


@pytest.mark.parametrize("alpha", [1, 3])
def test_kad_lazy_matches_eager(alpha):
    net = W.population(3000, 95)
    p = kad_params(lookupParallelRpcs=alpha)
    e = OracleNet("kademlia", net.ids, net.xy, p)
    z = OracleNet("kademlia", net.ids, net.xy, p, lazy=True)
    for a, b in zip(e.kad_tables(), z.kad_tables()):
        assert np.array_equal(a, b)
    k1, s1 = W.lookups(net.ids, 2000, 96, node_ids=True)
    k2, s2 = W.lookups(net.ids, 2000, 97, node_ids=False)
    keys, src = np.concatenate([k1, k2]), np.concatenate([s1, s2])
    _same(e.route(keys, src, count_rpcs=True), z.route(keys, src, count_rpcs=True), ("hop_seq", "rpcs"))
    le = e.lookup_call(keys[:500], src[:500])
    lz = z.lookup_call(keys[:500], src[:500])
    for f in le:
        assert np.array_equal(le[f], lz[f]), f


def test_oracle_rejects_capacity_breaking_params():
    net = W.population(50, 98)
    with pytest.raises(RuntimeError):
        OracleNet("chord", net.ids, net.xy, chord_params(successorListSize=200))
    with pytest.raises(RuntimeError):
        OracleNet("kademlia", net.ids, net.xy, kad_params(s=30))
