"""Kademlia maintenance rounds on the CPU: the oracle's restatement of Kademlia::routingAdd and of a
synchronous refresh round (orc_kad_maintenance_round; Kademlia.cc:432-756, 1328-1420, 1591-1686)
against the independent Python reading (tests/refmodel.py KadMaint: its own tables, routingAdd,
refresh keys, findNode and message-level lookup simulation), and the round's fixed point.  CPU only."""
from __future__ import annotations

import numpy as np
import pytest

import refmodel
from kad_maint import partial_join
from oracle_lib import OracleNet, kad_params
from oversim_amd import workload as W

LOOKUP_CFG = dict(redundant=8, alpha=3, merge=True, strict=True, visit_once=True, accept_late_siblings=True,
                  use_all=False, new_on_timeout=False, new_on_response=False, finish_on_first_unchanged=False,
                  hop_max=50, rnd=True, rpc_timeout=1.5, lookup_timeout=10.0)


def _same_tables(o: OracleNet, m: refmodel.KadMaint, what: str):
    sib, cnt, nodes = o.kad_tables()
    s2, c2, n2 = (np.array(a, dtype=t) for a, t in zip(m.arrays(), (np.uint32, np.uint8, np.uint32)))
    bad = np.nonzero((sib != s2).any(axis=1))[0]
    assert len(bad) == 0, f"{what}: sibling tables differ at nodes {bad[:5]}"
    bad = np.nonzero((cnt != c2).any(axis=1) | (nodes != n2).any(axis=(1, 2)))[0]
    assert len(bad) == 0, f"{what}: buckets (members or LRU order) differ at nodes {bad[:5]}"


def test_routing_add_rules():
    """routingAdd one call at a time on a small network: both readings agree after every call --
    sibling insertion and preemption into the bucket, full buckets, LRU moves of alive handles."""
    net = W.population(300, 0x4b60)
    tabs, join = partial_join(net.ids, net.xy, 0.3, 3)
    o = OracleNet("kademlia", net.ids, net.xy, kad_params(), tables=tabs)
    m = refmodel.KadMaint(net.ids, tabs["siblings"], tabs["bucket_count"], tabs["bucket_nodes"])
    rng = np.random.default_rng(4)
    results = set()
    for i in range(4000):
        v = int(rng.integers(0, len(net.ids)))
        x = int(join[rng.integers(0, len(join))]) if i % 2 else int(rng.integers(0, len(net.ids)))
        alive = bool(rng.integers(0, 2))
        r1 = o.routing_add(v, x, alive)
        r2 = m.routing_add(v, x, alive)
        assert r1 == int(r2), (i, v, x, alive)
        results.add(r1)
    assert results == {0, 1}
    _same_tables(o, m, "after 4000 routingAdds")


@pytest.mark.parametrize("alpha", [3, 1])
def test_round_matches_second_reading(alpha):
    """A joiners' round (sibling refresh only) and a round of bucket + sibling refreshes of a node
    sample: identical tables (members and LRU order) from both readings."""
    net = W.population(400, 0x4b61)
    p = kad_params(lookupParallelRpcs=alpha)
    tabs, join = partial_join(net.ids, net.xy, 0.2, 5, p)
    o = OracleNet("kademlia", net.ids, net.xy, p, tables=tabs)
    m = refmodel.KadMaint(net.ids, tabs["siblings"], tabs["bucket_count"], tabs["bucket_nodes"])
    cfg = dict(LOOKUP_CFG, alpha=alpha)
    st = o.maintenance_round(join, flags=1)
    n = m.round(net.xy, [int(v) for v in join], [1] * len(join), cfg)
    assert st["lookups"] == n and st["changes"] > 0
    _same_tables(o, m, "joiners' round")
    sample = np.arange(1, len(net.ids), 9, dtype=np.uint32)
    st = o.maintenance_round(sample, flags=3)
    n = m.round(net.xy, [int(v) for v in sample], [3] * len(sample), cfg)
    assert st["lookups"] == n
    _same_tables(o, m, "bucket + sibling refresh round")


def test_rounds_reach_the_snapshot_siblings():
    """From a network where 10 % of the nodes just joined, full refresh rounds reach a fixed point
    (no membership change) whose sibling tables are the XOR-closest 5s nodes -- what the snapshot
    rule builds -- and whose buckets hold as many members as the snapshot's (which ones depends on
    the order nodes were learned; the snapshot samples them)."""
    net = W.population(2000, 0x4b51)
    tabs, join = partial_join(net.ids, net.xy, 0.1, 7)
    o = OracleNet("kademlia", net.ids, net.xy, kad_params(), tables=tabs)
    assert o.maintenance_round(join, flags=1)["changes"] > 0
    for r in range(6):
        st = o.maintenance_round()
        if st["changes"] == 0:
            break
    assert st["changes"] == 0, "no fixed point within 6 rounds"
    sib, cnt, _ = o.kad_tables()
    s2, c2, _ = OracleNet("kademlia", net.ids, net.xy, kad_params()).kad_tables()
    assert all(set(a[a != 0xFFFFFFFF]) == set(b[b != 0xFFFFFFFF]) for a, b in zip(sib, s2))
    assert np.mean(cnt == c2) > 0.9999
