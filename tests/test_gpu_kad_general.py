"""Kademlia variants on the GPU (K2g, oversim_amd/csrc/kad_general.hip) through the CSR table import
(ovs_kad_load_tables_csr): b = 2, 3, 4 (routingBucketIndex's b-bit digits, numBuckets =
(2^b - 1) * (160 / b), Kademlia.cc:176, 357-382), bucketType nr128 (final buckets of up to 128,
routingBucketSize 384-411) and nkademlia (no per-bucket maximum under globalNodeLimit, 620-664),
plus b = 1 kademlia tables through the same path.  Tables come from the oracle (snapshot rule, or
maintenance rounds after a partial join for nkademlia) and are then made non-converged (bucket
members dropped, LRU order shuffled, some sibling tables cut); the engine is compared with the
oracle run over the same tables: findNode and the siblings flag, one-way lookups (alpha 1, 3, 8)
with hop sequences and RPC counts, LookupCalls."""
from __future__ import annotations

import numpy as np
import pytest

from kad_maint import partial_join
from oracle_lib import OracleNet, kad_params
from oversim_amd import KbrEngine, KbrError, Params, workload as W

pytestmark = pytest.mark.gpu
FIELDS = ("responsible", "hops", "status", "one_way_hops", "latency_ns")
NONE = 0xFFFFFFFF

VARIANTS = {
    "b1": dict(b=1),
    "b2": dict(b=2),
    "b3": dict(b=3),
    "b4": dict(b=4),
    "nr128": dict(bucketType=2),
    "nkademlia": dict(bucketType=1),
}


def _perturb(sib, off, nodes, rng, s: int = 8):
    """~30 % of the bucket members dropped, buckets shuffled (LRU order), a quarter of the sibling
    tables cut to 3..5s-1 entries (the cut siblings forgotten), the rest shuffled."""
    sib = sib.copy()
    new_off = np.zeros_like(off)
    out = []
    for j in range(len(off) - 1):
        seg = [int(x) for x in nodes[off[j]:off[j + 1]] if rng.random() > 0.3]
        rng.shuffle(seg)
        out += seg
        new_off[j + 1] = len(out)
    S5 = 5 * s
    for v in range(len(sib)):
        row = [int(x) for x in sib[v] if x != NONE]
        if rng.random() < 0.25 and len(row) > 3:
            row = row[:int(rng.integers(3, len(row)))]
        else:
            rng.shuffle(row)
        sib[v, :] = NONE
        sib[v, :len(row)] = row
    assert sib.shape[1] == S5
    return sib, new_off, np.array(out, dtype=np.uint32)


def _variant_tables(name: str, n: int = 2500, seed: int = 0x6b20):
    net = W.population(n, seed)
    p = kad_params(**VARIANTS[name])
    rng = np.random.default_rng(seed + 7)
    if name == "nkademlia":
        tabs, join = partial_join(net.ids, net.xy, 0.3, seed, p, csr=True)
        o = OracleNet("kademlia", net.ids, net.xy, p, tables=tabs)
        o.maintenance_round(join, flags=1)
        o.maintenance_round(np.arange(0, n, 3, dtype=np.uint32), flags=3)
        sib, off, nodes = o.kad_tables_csr()
        assert np.diff(off).max() > 8          # buckets past k
        return net, dict(siblings=sib, bucket_off=off, bucket_nodes=nodes)
    sib, off, nodes = OracleNet("kademlia", net.ids, net.xy, p).kad_tables_csr()
    sib, off, nodes = _perturb(sib, off, nodes, rng)
    return net, dict(siblings=sib, bucket_off=off, bucket_nodes=nodes)


_CACHE: dict = {}


def _tables(name):
    if name not in _CACHE:
        _CACHE[name] = _variant_tables(name)
    return _CACHE[name]


def _load(engine: KbrEngine, name, **p):
    net, t = _tables(name)
    engine.set_params(Params.kademlia().replace(**VARIANTS[name], **p))
    engine.kad_load_tables_csr(net.ids, net.xy, t["siblings"], t["bucket_off"], t["bucket_nodes"])
    return net, t, OracleNet("kademlia", net.ids, net.xy, kad_params(**VARIANTS[name], **p), tables=t)


@pytest.mark.parametrize("name", list(VARIANTS))
def test_csr_round_trip(engine: KbrEngine, name):
    net, t, _ = _load(engine, name)
    sib, off, nodes = engine.kad_tables_csr()
    assert np.array_equal(off, t["bucket_off"].astype(np.uint64))
    assert np.array_equal(nodes, t["bucket_nodes"])
    for v in range(net.n):
        assert sorted(x for x in sib[v] if x != NONE) == sorted(int(x) for x in t["siblings"][v] if x != NONE)


@pytest.mark.parametrize("name", list(VARIANTS))
def test_find_node_matches_oracle(engine: KbrEngine, name):
    net, t, o = _load(engine, name)
    rng = np.random.default_rng(11)
    node = rng.integers(0, net.n, 1500).astype(np.uint32)
    keys = np.concatenate([W.random_keys(1000, rng), net.ids[rng.integers(0, net.n, 500)]])
    for nr, ns in ((8, 1), (3, 1), (8, 8), (16, 3), (8, -1), (40, -1)):
        got, cntg, sibg = engine.findNode(node, keys, nr, ns, max_out=max(nr, ns, 16))
        for i in range(len(node)):
            ref, flag = o.find_node(int(node[i]), keys[i], nr, ns)
            assert list(got[i, :cntg[i]]) == [int(x) for x in ref], (name, nr, ns, i)
            if ns >= 0:     # an exhaustive call (-1) carries no siblings flag (BaseOverlay.cc:1857-1871)
                assert bool(sibg[i]) == flag, (name, nr, ns, i)


@pytest.mark.parametrize("name", list(VARIANTS))
@pytest.mark.parametrize("alpha", [1, 3, 8])
def test_route_matches_oracle(engine: KbrEngine, name, alpha):
    net, t, o = _load(engine, name, lookupParallelRpcs=alpha)
    k1, s1 = W.lookups(net.ids, 2000, 402, node_ids=True)
    k2, s2 = W.lookups(net.ids, 2000, 403, node_ids=False)
    keys, src = np.concatenate([k1, k2]), np.concatenate([s1, s2])
    g = engine.lookup(keys, src, record_hops=True, count_rpcs=True)
    r = o.route(keys, src, record_hops=True, count_rpcs=True)
    for f in FIELDS + ("rpcs",):
        bad = np.nonzero(g[f].astype(np.int64) != r[f].astype(np.int64))[0]
        assert len(bad) == 0, (name, f, bad[:8], g[f][bad[:8]], r[f][bad[:8]])
    assert np.array_equal(g["hop_seq"], r["hop_seq"])
    assert (g["status"] == 0).mean() > 0.9


@pytest.mark.parametrize("name", ["b2", "b4", "nr128", "nkademlia"])
@pytest.mark.parametrize("alpha,ns", [(1, -1), (3, 3), (3, 0)])
def test_lookup_call_matches_oracle(engine: KbrEngine, name, alpha, ns):
    net, t, o = _load(engine, name, lookupParallelRpcs=alpha)
    keys, src = W.lookups(net.ids, 2000, 404 + alpha, node_ids=True)
    g = engine.lookupCall(keys, src, ns)
    r = o.lookup_call(keys, src, ns)
    for f in ("num_siblings", "hops", "status", "is_valid", "latency_ns", "siblings"):
        assert np.array_equal(np.asarray(g[f]).astype(np.int64), np.asarray(r[f]).astype(np.int64)), (name, f)


def test_kademlia_lookup_large(engine: KbrEngine):
    """KademliaLarge-style k = 16 / lookupRedundantNodes = 16 on b = 2 tables (the 16-entry K2g)."""
    net = W.population(2000, 0x6b30)
    p = dict(b=2, k=16)
    sib, off, nodes = OracleNet("kademlia", net.ids, net.xy, kad_params(**p)).kad_tables_csr()
    engine.set_params(Params.kademlia().replace(**p, lookupRedundantNodes=16))
    engine.kad_load_tables_csr(net.ids, net.xy, sib, off, nodes)
    o = OracleNet("kademlia", net.ids, net.xy, kad_params(**p, lookupRedundantNodes=16),
                  tables=dict(siblings=sib, bucket_off=off, bucket_nodes=nodes))
    keys, src = W.lookups(net.ids, 3000, 405, node_ids=False)
    g = engine.lookup(keys, src, record_hops=True, count_rpcs=True)
    r = o.route(keys, src, record_hops=True, count_rpcs=True)
    for f in FIELDS + ("rpcs",):
        assert np.array_equal(g[f].astype(np.int64), r[f].astype(np.int64)), f
    assert np.array_equal(g["hop_seq"], r["hop_seq"])


def test_rejects_broken_tables(engine: KbrEngine):
    net, t = _tables("b2")
    engine.set_params(Params.kademlia().replace(b=2))
    nb = engine.kad_num_buckets()
    assert nb == 240
    v = 23
    off, nodes = t["bucket_off"], t["bucket_nodes"].copy()
    row = off[v * nb:(v + 1) * nb + 1]
    m = int(np.nonzero(np.diff(row))[0][-1])
    nodes[off[v * nb + m]] = v                                  # the node in its own bucket
    with pytest.raises(KbrError, match="node 23"):
        engine.kad_load_tables_csr(net.ids, net.xy, t["siblings"], off, nodes)
    # a member moved to another digit bucket of its layer (one with room): routingBucketIndex differs
    sizes = np.diff(row)
    m2 = next(q for q in range(3 * (m // 3), 3 * (m // 3) + 3) if q != m and sizes[q] < 8)
    nodes = t["bucket_nodes"].copy()
    a = int(off[v * nb + m])
    x = int(nodes[a])
    new_nodes = np.delete(nodes, a)
    new_off = off.copy()
    new_off[v * nb + m + 1:] -= 1
    ins = int(new_off[v * nb + m2])
    new_nodes = np.insert(new_nodes, ins, x)
    new_off[v * nb + m2 + 1:] += 1
    with pytest.raises(KbrError, match="wrong bucket"):
        engine.kad_load_tables_csr(net.ids, net.xy, t["siblings"], new_off, new_nodes)
    # kademlia buckets hold at most k: a 9th member is refused
    engine.set_params(Params.kademlia().replace(b=2, k=4))
    with pytest.raises(KbrError, match="routingBucketSize"):
        engine.kad_load_tables_csr(net.ids, net.xy, t["siblings"], t["bucket_off"], t["bucket_nodes"])


def test_unsupported_on_general_tables(engine: KbrEngine):
    net, t, _ = _load(engine, "b2")
    keys, src = W.lookups(net.ids, 10, 406)
    engine.set_params(Params.kademlia().replace(b=2, routingType=3))
    with pytest.raises(KbrError, match="iterative"):
        engine.lookup(keys, src)
    engine.set_params(Params.kademlia().replace(b=2))
    with pytest.raises(KbrError, match="160-bucket"):
        engine.kad_maintenance_round(np.arange(4, dtype=np.uint32))
    # nr128 with b > 1 is refused (routingBucketSize overflows past index 159)
    with KbrEngine(0) as e2:
        e2.set_params(Params.kademlia().replace(b=2, bucketType=2))
        with pytest.raises(KbrError, match="nr128"):
            e2.kad_load_tables_csr(net.ids, net.xy, t["siblings"], t["bucket_off"], t["bucket_nodes"])
