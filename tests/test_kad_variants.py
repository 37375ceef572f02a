"""The fork's Kademlia variants on the CPU: b > 1 (numBuckets = (2^b - 1) * (160 / b), b-bit digits in
routingBucketIndex, Kademlia.cc:176, 357-382, and the digit loop of the bucket refresh, 1631-1676)
and the bucketType variants (nr128: bigger final buckets, nkademlia: buckets unbounded under a
global table limit; 135-151, 384-411, 620-664).  The oracle (oracle/ovs_oracle.c) against the
independent Python reading (tests/refmodel.py): findNode, one-way lookups, routingAdd and
maintenance rounds.  CPU only."""
from __future__ import annotations

import numpy as np
import pytest

import refmodel
from kad_maint import partial_join
from oracle_lib import OracleNet, kad_params
from oversim_amd import workload as W

VARIANTS = {
    "b2": dict(b=2),
    "b3": dict(b=3),
    "b4": dict(b=4),
    "nr128": dict(bucketType=2),
    "nr128_e40": dict(bucketType=2, extraNodesFinalBucket=40),
}


def _tables(o: OracleNet, p) -> refmodel.KadTables:
    sib, off, nodes = o.kad_tables_csr()
    nb = o.num_buckets()
    buckets = []
    for v in range(o.n):
        row = {}
        for m in range(nb):
            a, z = int(off[v * nb + m]), int(off[v * nb + m + 1])
            if z > a:
                row[m] = [int(x) for x in nodes[a:z]]
        buckets.append(row)
    return refmodel.KadTables(o.ids, sib, None, None, k=p.k, s=p.s, b=p.b, buckets=buckets)


def test_bucket_index_and_size_rules():
    """routingBucketIndex / routingBucketSize / numBuckets against a direct reading."""
    p = kad_params()
    assert [OracleNet.__new__(OracleNet) is not None]
    from oracle_lib import lib
    import ctypes as C
    for b in (1, 2, 3, 4, 5):
        q = p.replace(b=b)
        assert lib().orc_kad_num_buckets(C.byref(q)) == refmodel.kad_num_buckets(b)
    q = p.replace(bucketType=2)
    sizes = {m: lib().orc_kad_bucket_size(C.byref(q), m) for m in range(160)}
    assert sizes[159] == 128 and sizes[158] == 64 and sizes[157] == 32 and sizes[156] == 16 and sizes[155] == 8
    assert all(sizes[m] == refmodel.kad_bucket_size(m, 8, 2) for m in range(160))
    assert lib().orc_kad_bucket_size(C.byref(p.replace(bucketType=1)), 3) == 0
    # b = 3: bit 0 is never a digit (positions 157, 154, ..., 1), so a distance of 1 has no bucket
    assert refmodel.kad_bucket_index(1, 3) == -1 and refmodel.kad_bucket_index(2, 3) == 0
    assert refmodel.kad_bucket_index(1 << 159, 2) == 79 * 3 + 1
    # nr128 with b > 1 is refused (routingBucketSize indexes as if b = 1; sizes overflow past 160)
    with pytest.raises(Exception, match="nr128"):
        OracleNet("kademlia", *_small(), kad_params(b=2, bucketType=2))


def _small():
    net = W.population(64, 5)
    return net.ids, net.xy


@pytest.mark.parametrize("name", list(VARIANTS))
def test_find_node_agrees(name):
    net = W.population(1200, 0x4b80)
    p = kad_params(**VARIANTS[name])
    o = OracleNet("kademlia", net.ids, net.xy, p)
    T = _tables(o, p)
    rng = np.random.default_rng(3)
    keys, _ = W.lookups(net.ids, 300, 9, node_ids=False)
    for i in range(300):
        c = int(rng.integers(0, len(net.ids)))
        key = keys[i] if i % 3 else net.ids[int(rng.integers(0, len(net.ids)))]
        for nr, ns in ((8, 1), (8, -1), (3, 3), (20, -1)):
            got, flag = o.find_node(c, key, nr, ns)
            want = T.find_node(c, refmodel.to_int(key), nr, ns)
            assert [int(x) for x in got] == want, (name, i, nr, ns)


@pytest.mark.parametrize("name", ["b2", "b4", "nr128"])
def test_lookups_agree(name):
    net = W.population(1000, 0x4b81)
    p = kad_params(lookupParallelRpcs=3, **VARIANTS[name])
    o = OracleNet("kademlia", net.ids, net.xy, p)
    sim = refmodel.KadLookupSim(_tables(o, p), net.xy, redundant=8, alpha=3, k=p.k)
    k1, s1 = W.lookups(net.ids, 150, 21, node_ids=True)
    k2, s2 = W.lookups(net.ids, 150, 22, node_ids=False)
    keys, src = np.concatenate([k1, k2]), np.concatenate([s1, s2])
    r = o.route(keys, src, record_hops=True, count_rpcs=True)
    for i in range(len(keys)):
        m = sim.run(keys[i], int(src[i]))
        for f in ("responsible", "hops", "status", "latency_ns", "rpcs"):
            assert int(r[f][i]) == int(m[f]), (name, i, f)
        assert [int(x) for x in r["hop_seq"][i] if x != 0xFFFFFFFF] == m["hop_seq"], (name, i)


def _maint(net, tabs, p):
    return refmodel.KadMaint(net.ids, tabs["siblings"], k=p.k, s=p.s, b=p.b, bucket_type=p.bucketType,
                             node_limit=p.globalNodeLimit, extra=p.extraNodesFinalBucket,
                             bucket_off=tabs["bucket_off"], bucket_nodes=tabs["bucket_nodes"])


def _same(o: OracleNet, m: refmodel.KadMaint, what):
    s1, o1, n1 = o.kad_tables_csr()
    s2, o2, n2 = m.csr()
    assert np.array_equal(s1, np.array(s2, dtype=np.uint32)), f"{what}: sibling tables"
    assert np.array_equal(o1, np.array(o2, dtype=np.uint64)), f"{what}: bucket sizes"
    assert np.array_equal(n1, np.array(n2, dtype=np.uint32)), f"{what}: bucket members / LRU order"


@pytest.mark.parametrize("name,kw", [("b2", dict(b=2)), ("nr128", dict(bucketType=2)),
                                     ("nkademlia", dict(bucketType=1, globalNodeLimit=60)),
                                     ("b3_nkad", dict(b=3, bucketType=1, globalNodeLimit=80))])
def test_rounds_agree(name, kw):
    """routingAdd and two maintenance rounds (joiners, then a node sample) from both readings."""
    net = W.population(300, 0x4b82)
    p = kad_params(**kw)
    tabs, join = partial_join(net.ids, net.xy, 0.2, 4, p, csr=True)
    o = OracleNet("kademlia", net.ids, net.xy, p, tables=tabs)
    m = _maint(net, tabs, p)
    _same(o, m, f"{name} start")
    cfg = dict(redundant=8, alpha=3)
    st = o.maintenance_round(join, flags=1)
    m.round(net.xy, [int(v) for v in join], [1] * len(join), cfg)
    assert st["changes"] > 0
    _same(o, m, f"{name} joiners' round")
    sample = np.arange(2, len(net.ids), 7, dtype=np.uint32)
    o.maintenance_round(sample, flags=3)
    m.round(net.xy, [int(v) for v in sample], [3] * len(sample), cfg)
    _same(o, m, f"{name} refresh round")
    if kw.get("bucketType") == 1:      # nkademlia: buckets past k, tables at the global limit
        _, off, _ = o.kad_tables_csr()
        sizes = np.diff(off)
        assert sizes.max() > 8
