"""Kademlia refresh lookups on the GPU (K2x, ovs_kad_refresh_batch / ovs_kad_refresh_keys) against
the oracle: Kademlia::handleBucketRefreshTimerExpired (Kademlia.cc:1591-1686) with
exhaustiveRefresh = true -- the bucket-refresh keys self ^ 2^i and EXHAUSTIVE_ITERATIVE_ROUTING
lookups with redundantNodes = bucketRefreshNodes (k = 8) or siblingRefreshNodes (5s = 40),
IterativeLookup.cc:133-244, 488-585, 714-781, 803-1170.  Every field is compared bit-exactly:
validity, status, hops, FindNodeCall count, duration in ns, the result (siblings) and the
responders with their RTTs, which feed the host's routingAdd."""
from __future__ import annotations

import numpy as np
import pytest

from oversim_amd import KbrEngine, KbrError, Params, workload as W
from oracle_lib import OracleNet, kad_params
from test_gpu_kad_tables import _explicit_tables

pytestmark = pytest.mark.gpu
FIELDS = ("num_siblings", "hops", "status", "is_valid", "latency_ns")


def _params(**kw) -> Params:
    p = Params.kademlia()
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def _compare(r, o, R, what):
    for f in FIELDS:
        bad = np.nonzero(r[f] != o[f])[0]
        assert len(bad) == 0, f"{what}: {f} differs at {bad[:5]}: gpu {r[f][bad[:5]]} oracle {o[f][bad[:5]]}"
    assert np.array_equal(r["rpcs"], o["rpcs"]), f"{what}: rpcs"
    assert np.array_equal(r["siblings"][:, :R], o["siblings"]), f"{what}: siblings"
    assert np.array_equal(r["responders"], o["responders"]), f"{what}: responders"
    assert np.array_equal(r["rtt_ns"], o["rtt_ns"]), f"{what}: rtt"


@pytest.fixture(scope="module")
def net():
    return W.population(2000, 0x5EF)


def test_refresh_keys_match_oracle(engine, net):
    engine.set_params(Params.kademlia())
    engine.kad_load(net.ids, net.xy)
    o = OracleNet("kademlia", net.ids, net.xy, kad_params())
    nodes = np.arange(0, len(net.ids), 13, dtype=np.uint32)
    k1, s1 = engine.kad_refresh_keys(nodes)
    k2, s2 = o.refresh_keys(nodes)
    assert len(k1) > 10 * len(nodes)
    assert np.array_equal(k1, k2) and np.array_equal(s1, s2)
    rng = np.random.default_rng(5)
    stale = rng.integers(0, 1 << 32, size=(len(nodes), 5), dtype=np.uint64).astype(np.uint32)
    k1, s1 = engine.kad_refresh_keys(nodes, stale)
    k2, s2 = o.refresh_keys(nodes, stale)
    assert np.array_equal(k1, k2) and np.array_equal(s1, s2)


VARIANTS = {
    "a3": dict(lookupParallelRpcs=3),
    "a1": dict(lookupParallelRpcs=1),
    "a2": dict(lookupParallelRpcs=2),
    "a4": dict(lookupParallelRpcs=4),
    # RPC timeouts (RTTs reach ~1.3 s on these coordinates): dead nodes leave nextHops
    "a3_rpcto": dict(lookupParallelRpcs=3, rpcUdpTimeout=0.35),
    "a3_rpcto_newto": dict(lookupParallelRpcs=3, rpcUdpTimeout=0.35, lookupNewRpcOnEveryTimeout=1),
    "a2_lookupto": dict(lookupParallelRpcs=2, lookupTimeout=0.9),
    "a3_hcm12": dict(lookupParallelRpcs=3, hopCountMax=12),
    "a3_newresp": dict(lookupParallelRpcs=3, lookupNewRpcOnEveryResponse=1),
    "a3_trunc": dict(lookupParallelRpcs=3, simtimeRound=0),
    # the 8-slot instantiations (lookupParallelRpcs 5..8; maidsafe.ini:18-19 sets 8)
    "a8": dict(lookupParallelRpcs=8),
    "a6_rpcto": dict(lookupParallelRpcs=6, rpcUdpTimeout=0.35),
}


@pytest.mark.parametrize("name", list(VARIANTS))
def test_refresh_lookups_match_oracle(engine, net, name):
    kw = VARIANTS[name]
    engine.set_params(_params(**kw))
    engine.kad_load(net.ids, net.xy)
    o = OracleNet("kademlia", net.ids, net.xy, kad_params(**kw))
    nodes = np.arange(3, len(net.ids), 37, dtype=np.uint32)
    keys, src = o.refresh_keys(nodes)
    # the bucket refreshes (R = k) and the sibling-table refreshes of the nodes' own keys (R = 5s)
    for R, K, S in ((8, keys, src), (40, net.ids[nodes], nodes)):
        r = engine.kad_refresh(K, S, R)
        e = o.exhaustive(K, S, R)
        _compare(r, e, R, f"{name} R={R}")
    if "rpcto" in name:
        assert (e["rpcs"] > (e["responders"] != 0xFFFFFFFF).sum(axis=1)).any(), "no call timed out"


def test_refresh_explicit_tables(engine):
    """Non-converged tables (partial buckets, short sibling tables, LRU order)."""
    net, t = _explicit_tables(3000, 303)
    p = dict(lookupParallelRpcs=3)
    engine.set_params(_params(**p))
    engine.kad_load_tables(net.ids, net.xy, t["siblings"], t["bucket_count"], t["bucket_nodes"])
    o = OracleNet("kademlia", net.ids, net.xy, kad_params(**p), tables=t)
    nodes = np.arange(1, len(net.ids), 41, dtype=np.uint32)
    keys, src = o.refresh_keys(nodes)
    k1, s1 = engine.kad_refresh_keys(nodes)
    assert np.array_equal(k1, keys) and np.array_equal(s1, src)
    for R, K, S in ((8, keys, src), (40, net.ids[nodes], nodes), (5, keys[::3], src[::3])):
        _compare(engine.kad_refresh(K, S, R), o.exhaustive(K, S, R), R, f"explicit R={R}")


def test_refresh_large_network_sample(engine):
    """2^18 nodes, alpha = 3: the refresh round of 512 nodes (~9k lookups) against the lazy-table
    oracle; every successful bucket refresh returns the R XOR-closest nodes of its key."""
    n = 1 << 18
    net = W.population(n, 0x18EF)
    engine.set_params(_params(lookupParallelRpcs=3))
    engine.kad_load(net.ids, net.xy)
    o = OracleNet("kademlia", net.ids, net.xy, kad_params(lookupParallelRpcs=3), lazy=True)
    nodes = np.random.default_rng(9).choice(n, 512, replace=False).astype(np.uint32)
    keys, src = engine.kad_refresh_keys(nodes)
    r = engine.kad_refresh(keys, src, 8)
    e = o.exhaustive(keys, src, 8)
    _compare(r, e, 8, "2^18")
    assert (r["status"] == 0).mean() > 0.99
    # the result of a successful exhaustive lookup is the 8 XOR-closest nodes (sampled check)
    ids = [int(sum(int(w[i]) << (32 * i) for i in range(5))) for w in net.ids]
    for i in (0, len(keys) // 2, len(keys) - 1):
        if r["status"][i] != 0:
            continue
        K = sum(int(keys[i][j]) << (32 * j) for j in range(5))
        assert list(r["siblings"][i]) == sorted(range(n), key=lambda v: ids[v] ^ K)[:8], i


@pytest.mark.parametrize("name", ["default", "a3_rpcto", "a2"])
def test_refresh_without_responders_device(engine, net, name):
    """The device-pointer refresh with no responder record (the bench's call): the responders stay
    in LDS, and the default configuration (R = k = 8, alpha 3, hopCountMax 50, strict, visitOnlyOnce)
    takes K2x's compile-time-configured instantiation (kad_refresh.hip kad_def_cfg).  Result,
    status, hops, duration and FindNodeCall count equal the oracle's."""
    import torch
    from oversim_amd.kbr import LOOKUP_OUT_DTYPE
    kw = {} if name == "default" else VARIANTS[name]
    engine.set_params(_params(**kw))
    engine.kad_load(net.ids, net.xy)
    o = OracleNet("kademlia", net.ids, net.xy, kad_params(**kw))
    keys, src = o.refresh_keys(np.arange(0, len(net.ids), 7, dtype=np.uint32))
    e = o.exhaustive(keys, src, 8)
    m = len(keys)
    dev = torch.device("cuda", 0)
    dk = torch.from_numpy(np.ascontiguousarray(keys).view(np.int32)).to(dev)
    ds = torch.from_numpy(np.ascontiguousarray(src).view(np.int32)).to(dev)
    dout = torch.empty((m, 16), dtype=torch.uint8, device=dev)
    dsib = torch.empty((m, 8), dtype=torch.int32, device=dev)
    drpc = torch.empty(m, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    engine.kad_refresh_device(dk.data_ptr(), ds.data_ptr(), m, 8, dout.data_ptr(), dsib.data_ptr(), drpc.data_ptr())
    torch.cuda.synchronize()
    r = dout.cpu().numpy().reshape(-1).view(LOOKUP_OUT_DTYPE)
    for f in FIELDS:
        bad = np.nonzero(r[f] != e[f])[0]
        assert len(bad) == 0, f"{name}: {f} differs at {bad[:5]}: gpu {r[f][bad[:5]]} oracle {e[f][bad[:5]]}"
    assert np.array_equal(drpc.cpu().numpy().view(np.uint32), e["rpcs"]), f"{name}: rpcs"
    assert np.array_equal(dsib.cpu().numpy().view(np.uint32), e["siblings"]), f"{name}: siblings"


def test_refresh_rejects_unsupported(engine, net):
    engine.set_params(_params(lookupParallelRpcs=3))
    engine.kad_load(net.ids, net.xy)
    keys, src = net.ids[:4], np.arange(4, dtype=np.uint32)
    with pytest.raises(KbrError):
        engine.kad_refresh(keys, src, 65)
    engine.set_params(_params(lookupParallelRpcs=3, lookupStrictParallelRpcs=0))
    with pytest.raises(KbrError):
        engine.kad_refresh(keys, src, 8)


def test_exhaustive_find_node_calls(engine, net):
    """findNodeRpc of an exhaustive call: findNode(key, R, -1) -- resultSize R, no sibling flag."""
    engine.set_params(Params.kademlia())
    engine.kad_load(net.ids, net.xy)
    o = OracleNet("kademlia", net.ids, net.xy, kad_params())
    rng = np.random.default_rng(21)
    node = rng.integers(0, len(net.ids), 300).astype(np.uint32)
    keys = np.concatenate([W.random_keys(150, rng), net.ids[node[150:]]])
    for R in (8, 16):
        got, cnt, sib = engine.findNode(node, keys, R, -1, max_out=16)
        assert not sib.any()
        for i in range(len(node)):
            exp = o.find_node(int(node[i]), keys[i], R, -1)[0]
            assert list(got[i, :cnt[i]]) == list(exp), (R, i)


@pytest.mark.parametrize("alpha", [1, 3])
def test_exhaustive_routing_type(engine, net, alpha):
    """routingType = "exhaustive-iterative" (BaseOverlay.cc:123-124, 1434-1442) through the one-way
    route (numSiblings 1: route message to the closest node the lookup found) and LookupCalls
    (numSiblings = s), both on K2x."""
    kw = dict(lookupParallelRpcs=alpha, routingType=3)
    engine.set_params(_params(**kw))
    engine.kad_load(net.ids, net.xy)
    o = OracleNet("kademlia", net.ids, net.xy, kad_params(**kw))
    k1, s1 = W.lookups(net.ids, 1500, 77, node_ids=False)
    k2, s2 = W.lookups(net.ids, 500, 78, node_ids=True)
    keys, src = np.concatenate([k1, k2]), np.concatenate([s1, s2])
    r = engine.lookup(keys, src, record_hops=True, count_rpcs=True)
    e = o.route(keys, src, record_hops=True, count_rpcs=True)
    for f in ("responsible", "hops", "status", "one_way_hops", "latency_ns", "rpcs"):
        assert np.array_equal(r[f], e[f]), f
    assert np.array_equal(r["hop_seq"], e["hop_seq"])
    c = engine.lookupCall(keys, src, 8)
    ce = o.lookup_call(keys, src, 8)
    for f in FIELDS:
        assert np.array_equal(c[f], ce[f]), f
    assert np.array_equal(c["siblings"], ce["siblings"])
