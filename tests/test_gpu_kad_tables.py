"""Explicit Kademlia tables through the drop-in boundary (ovs_kad_load_tables): the k-buckets a
running OverSim node holds (Kademlia::routingTable, LRU-ordered buckets filled by routingAdd,
Kademlia.cc:432-756; Kademlia::siblingTable, KademliaBucket.h:30-69) rather than the snapshot
rule.  Tables are derived from the snapshot and then made non-converged -- partially filled
buckets, sibling tables shorter than 5s with the evicted siblings moved to their buckets or
forgotten, shuffled (LRU) bucket order -- and the HIP engine is compared with the oracle run over
the same tables: findNode, the siblings flag, one-way lookups (alpha 1 and 3) and LookupCalls."""
from __future__ import annotations

import numpy as np
import pytest

from oversim_amd import KbrEngine, KbrError, Params, workload as W
from oracle_lib import OracleNet, kad_params

pytestmark = pytest.mark.gpu
FIELDS = ("responsible", "hops", "status", "one_way_hops", "latency_ns")
NONE = 0xFFFFFFFF


def _msb_xor(a, b) -> int:
    x = 0
    for i in range(5):
        x |= (int(a[i]) ^ int(b[i])) << (32 * i)
    return x.bit_length() - 1


def _explicit_tables(n: int, seed: int, k: int = 8, s: int = 8):
    """Non-converged tables from the snapshot: ~30 % of bucket entries dropped, buckets shuffled,
    a quarter of the sibling tables cut to 3..39 entries (the cut siblings go to their bucket when
    it has room, else are forgotten)."""
    net = W.population(n, seed)
    rng = np.random.default_rng(seed + 1)
    sib, cnt, nodes = OracleNet("kademlia", net.ids, net.xy, kad_params(k=k, s=s)).kad_tables()
    sib, cnt, nodes = sib.copy(), cnt.copy(), nodes.copy()
    S5 = 5 * s
    for v in range(n):
        for m in np.nonzero(cnt[v])[0]:
            c = int(cnt[v, m])
            keep = [x for x in nodes[v, m, :c] if rng.random() > 0.3]
            rng.shuffle(keep)
            nodes[v, m, :] = NONE
            nodes[v, m, :len(keep)] = keep
            cnt[v, m] = len(keep)
        if rng.random() < 0.25:
            row = [int(x) for x in sib[v] if x != NONE]
            # the oracle's export is XOR-sorted: keep the closest, evict the rest
            cut = int(rng.integers(3, S5))
            evicted = row[cut:]
            sib[v, :] = NONE
            sib[v, :cut] = row[:cut]
            for x in evicted:
                m = _msb_xor(net.ids[x], net.ids[v])
                if cnt[v, m] < k and rng.random() < 0.7:
                    nodes[v, m, cnt[v, m]] = x
                    cnt[v, m] += 1
        else:
            row = [int(x) for x in sib[v] if x != NONE]
            rng.shuffle(row)            # any order: the engine and the oracle sort it like siblingTable
            sib[v, :] = NONE
            sib[v, :len(row)] = row
    return net, dict(siblings=sib, bucket_count=cnt, bucket_nodes=nodes)


@pytest.fixture(scope="module")
def tables():
    return _explicit_tables(3000, 301)


def _load(engine, net, t, **p):
    engine.set_params(Params.kademlia().replace(**p))
    engine.kad_load_tables(net.ids, net.xy, t["siblings"], t["bucket_count"], t["bucket_nodes"])


def test_tables_round_trip(engine: KbrEngine, tables):
    net, t = tables
    _load(engine, net, t)
    sib, cnt, nodes = engine.kad_tables()
    assert np.array_equal(cnt, t["bucket_count"])
    assert np.array_equal(nodes, t["bucket_nodes"])
    for v in range(net.n):
        assert sorted(x for x in sib[v] if x != NONE) == sorted(int(x) for x in t["siblings"][v] if x != NONE)


@pytest.mark.parametrize("nr,ns", [(8, 1), (3, 1), (8, 8), (8, 3)])
def test_find_node_matches_oracle(engine: KbrEngine, tables, nr, ns):
    net, t = tables
    _load(engine, net, t)
    o = OracleNet("kademlia", net.ids, net.xy, kad_params(), tables=t)
    rng = np.random.default_rng(7)
    node = rng.integers(0, net.n, 3000).astype(np.uint32)
    keys = np.concatenate([W.random_keys(1500, rng), net.ids[rng.integers(0, net.n, 1500)]])
    got, cntg, sibg = engine.findNode(node, keys, nr, ns)
    for i in range(len(node)):
        ref, flag = o.find_node(int(node[i]), keys[i], nr, ns)
        assert list(got[i, :cntg[i]]) == [int(x) for x in ref], (i, got[i, :cntg[i]], ref)
        assert bool(sibg[i]) == flag, i


@pytest.mark.parametrize("alpha", [1, 3])
def test_route_matches_oracle(engine: KbrEngine, tables, alpha):
    net, t = tables
    _load(engine, net, t, lookupParallelRpcs=alpha)
    o = OracleNet("kademlia", net.ids, net.xy, kad_params(lookupParallelRpcs=alpha), tables=t)
    k1, s1 = W.lookups(net.ids, 4000, 302, node_ids=True)
    k2, s2 = W.lookups(net.ids, 4000, 303, node_ids=False)
    keys, src = np.concatenate([k1, k2]), np.concatenate([s1, s2])
    g = engine.lookup(keys, src, record_hops=True, count_rpcs=True)
    r = o.route(keys, src, record_hops=True, count_rpcs=True)
    for f in FIELDS + ("rpcs",):
        bad = np.nonzero(g[f].astype(np.int64) != r[f].astype(np.int64))[0]
        assert len(bad) == 0, (f, bad[:8], g[f][bad[:8]], r[f][bad[:8]])
    assert np.array_equal(g["hop_seq"], r["hop_seq"])


@pytest.mark.parametrize("alpha,ns", [(1, -1), (3, 3)])
def test_lookup_call_matches_oracle(engine: KbrEngine, tables, alpha, ns):
    net, t = tables
    _load(engine, net, t, lookupParallelRpcs=alpha)
    o = OracleNet("kademlia", net.ids, net.xy, kad_params(lookupParallelRpcs=alpha), tables=t)
    keys, src = W.lookups(net.ids, 3000, 304 + alpha, node_ids=True)
    g = engine.lookupCall(keys, src, ns)
    r = o.lookup_call(keys, src, ns)
    for f in ("num_siblings", "hops", "status", "is_valid", "latency_ns", "siblings"):
        assert np.array_equal(np.asarray(g[f]).astype(np.int64), np.asarray(r[f]).astype(np.int64)), f


def test_rejects_broken_tables(engine: KbrEngine, tables):
    net, t = tables
    engine.set_params(Params.kademlia())
    bad = {k: v.copy() for k, v in t.items()}
    v = 17
    m = int(np.nonzero(bad["bucket_count"][v])[0][-1])
    bad["bucket_nodes"][v, m, 0] = v                          # the node in its own bucket
    with pytest.raises(KbrError, match="node 17"):
        engine.kad_load_tables(net.ids, net.xy, bad["siblings"], bad["bucket_count"], bad["bucket_nodes"])
    bad = {k: v.copy() for k, v in t.items()}
    x = int(bad["bucket_nodes"][v, m, 0])
    m2 = (m + 1) % 160 if bad["bucket_count"][v, (m + 1) % 160] < 8 else (m + 2) % 160
    bad["bucket_nodes"][v, m2, bad["bucket_count"][v, m2]] = x  # a member in the wrong bucket
    bad["bucket_count"][v, m2] += 1
    with pytest.raises(KbrError, match="wrong bucket|twice"):
        engine.kad_load_tables(net.ids, net.xy, bad["siblings"], bad["bucket_count"], bad["bucket_nodes"])
