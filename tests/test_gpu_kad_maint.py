"""Kademlia maintenance rounds on the GPU (ovs_kad_maintenance_round) against the oracle
(orc_kad_maintenance_round): the refresh lookups of Kademlia::handleBucketRefreshTimerExpired
(Kademlia.cc:1591-1686) routed by K2x on the device, Kademlia::routingAdd (432-756) applied on the
host for every FindNodeCall and FindNodeResponse (handleRpcCall / handleRpcResponse, 1328-1420) in
simulated-time order.  The tables after every round -- sibling tables, bucket members and their LRU
order -- and the round's counters are compared exactly; the rounds are run from a network where
some nodes just joined until they stop changing, and lookups over the converged tables are
compared with the oracle routing over the same tables."""
from __future__ import annotations

import numpy as np
import pytest

from kad_maint import partial_join
from oracle_lib import OracleNet, kad_params
from oversim_amd import KbrEngine, Params, workload as W

pytestmark = pytest.mark.gpu
STATS = ("lookups", "failed", "responses", "sib_changes", "bucket_changes", "lost", "replacement", "refreshed")
FIELDS = ("responsible", "hops", "status", "one_way_hops", "latency_ns")


def _params(**kw) -> Params:
    p = Params.kademlia()
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def _same(engine: KbrEngine, o: OracleNet, what: str):
    s1, c1, n1 = engine.kad_tables()
    s2, c2, n2 = o.kad_tables()
    bad = np.nonzero((s1 != s2).any(axis=1))[0]
    assert len(bad) == 0, f"{what}: sibling tables differ at {bad[:5]}"
    bad = np.nonzero((c1 != c2).any(axis=1) | (n1 != n2).any(axis=(1, 2)))[0]
    assert len(bad) == 0, f"{what}: buckets differ at {bad[:5]}"


def _round(engine, o, what, nodes=None, flags=None, stale=None):
    a = engine.kad_maintenance_round(nodes, flags, stale)
    b = o.maintenance_round(nodes, flags, stale)
    for f in STATS:
        assert a[f] == b[f], f"{what}: {f} gpu {a[f]} oracle {b[f]}"
    _same(engine, o, what)
    return a


@pytest.mark.parametrize("alpha", [3, 1, 8])
def test_rounds_match_oracle(engine, alpha):
    net = W.population(2000, 0x4b70 + alpha)
    kw = dict(lookupParallelRpcs=alpha)
    tabs, join = partial_join(net.ids, net.xy, 0.1, 11, kad_params(**kw))
    engine.set_params(_params(**kw))
    engine.kad_load_tables(net.ids, net.xy, tabs["siblings"], tabs["bucket_count"], tabs["bucket_nodes"])
    o = OracleNet("kademlia", net.ids, net.xy, kad_params(**kw), tables=tabs)
    st = _round(engine, o, "joiners' sibling refresh", join, 1)
    assert st["changes"] > 0
    rng = np.random.default_rng(alpha)
    sample = np.sort(rng.choice(len(net.ids), 300, replace=False)).astype(np.uint32)
    stale = rng.integers(0, 1 << 32, size=(len(sample), 5), dtype=np.uint64).astype(np.uint32)
    _round(engine, o, "sampled bucket refreshes", sample, 2, stale)
    _round(engine, o, "full round")


def test_rounds_converge_and_route(engine):
    """Config B's network (15 000 nodes, nodes_2d_15000 coordinates) with 10 % of its nodes just
    joined: full rounds until nothing changes; the fixed point's sibling tables are the XOR-closest
    5s, and 40 000 lookups over the converged tables equal the oracle's over the same tables."""
    net = W.population(15000, 0x4b41)
    tabs, join = partial_join(net.ids, net.xy, 0.1, 13)
    engine.set_params(Params.kademlia())
    engine.kad_load_tables(net.ids, net.xy, tabs["siblings"], tabs["bucket_count"], tabs["bucket_nodes"])
    st = engine.kad_maintenance_round(join, 1)
    assert st["changes"] > 0
    hist = [st["changes"]]
    for _ in range(8):
        st = engine.kad_maintenance_round()
        hist.append(st["changes"])
        if st["changes"] == 0:
            break
    assert hist[-1] == 0, f"no fixed point: {hist}"
    sib, cnt, nodes = engine.kad_tables()
    snap = OracleNet("kademlia", net.ids, net.xy, kad_params())
    s2, c2, _ = snap.kad_tables()
    assert all(set(a[a != 0xFFFFFFFF]) == set(b[b != 0xFFFFFFFF]) for a, b in zip(sib, s2))
    assert np.mean(cnt == c2) > 0.9999
    o = OracleNet("kademlia", net.ids, net.xy, kad_params(),
                  tables=dict(siblings=sib, bucket_count=cnt, bucket_nodes=nodes))
    k1, s1 = W.lookups(net.ids, 30000, 81, node_ids=True)
    k2, s2_ = W.lookups(net.ids, 10000, 82, node_ids=False)
    keys, src = np.concatenate([k1, k2]), np.concatenate([s1, s2_])
    for alpha in (1, 3):
        engine.set_params(_params(lookupParallelRpcs=alpha))
        engine.kad_load_tables(net.ids, net.xy, sib, cnt, nodes)
        o2 = OracleNet("kademlia", net.ids, net.xy, kad_params(lookupParallelRpcs=alpha),
                       tables=dict(siblings=sib, bucket_count=cnt, bucket_nodes=nodes))
        g = engine.lookup(keys, src, record_hops=True, count_rpcs=True)
        r = o2.route(keys, src, record_hops=True, count_rpcs=True)
        for f in FIELDS + ("rpcs",):
            bad = np.nonzero(g[f] != r[f])[0]
            assert len(bad) == 0, f"alpha={alpha} {f} differs at {bad[:5]}"
        assert np.array_equal(g["hop_seq"][:, :50], r["hop_seq"])
        assert np.all(g["status"][:30000] == 0)
    del o


def test_snapshot_is_a_fixed_point(engine):
    """The snapshot rule's tables (ovs_kad_load) do not change under a full round: every sibling
    table already holds the XOR-closest 5s and every bucket that is not full holds all of its
    subtree -- the snapshot is a state the reference's maintenance keeps."""
    net = W.population(1 << 14, 0x4b72)
    engine.set_params(Params.kademlia())
    engine.kad_load(net.ids, net.xy)
    before = engine.kad_tables()
    st = engine.kad_maintenance_round()
    assert st["changes"] == 0 and st["lookups"] > 10 * len(net.ids)
    after = engine.kad_tables()
    # the snapshot build stores sibling tables in index order, the round's rebuild XOR-sorted
    assert np.array_equal(np.sort(before[0], axis=1), np.sort(after[0], axis=1))
    assert np.array_equal(before[1], after[1])
    assert all(np.array_equal(np.sort(a, axis=-1), np.sort(b, axis=-1)) for a, b in zip(before[2], after[2]))


def test_failed_rebuild_leaves_no_tables(engine, monkeypatch):
    """a maintenance round whose table rebuild fails (forced here through the
    OVS_FAULT_INJECT test hook) must not leave the context routing on null or half-built device
    tables: the round reports the error, and every later call fails with OVS_ESTATE instead of
    launching a kernel."""
    from oversim_amd.kbr import KbrError
    net = W.population(2000, 0x4b79)
    tabs, join = partial_join(net.ids, net.xy, 0.1, 17)
    engine.set_params(Params.kademlia())
    engine.kad_load_tables(net.ids, net.xy, tabs["siblings"], tabs["bucket_count"], tabs["bucket_nodes"])
    monkeypatch.setenv("OVS_FAULT_INJECT", "kad_rebuild")
    with pytest.raises(KbrError, match="invariant"):
        engine.kad_maintenance_round(join, 1)
    monkeypatch.delenv("OVS_FAULT_INJECT")
    keys, src = W.lookups(net.ids, 256, 5, node_ids=True)
    with pytest.raises(KbrError, match="ESTATE|no network"):
        engine.lookup(keys, src)
    # the context is usable again after a reload
    engine.kad_load(net.ids, net.xy)
    assert np.all(engine.lookup(keys, src)["status"] == 0)
