"""[Config KademliaLarge] on the GPU: k = 16, lookupRedundantNodes = 16, s = 8, alpha = 1
(simulations/omnetpp.ini:113-126).  Buckets of up to 16 entries take two 96 B blocks
(KadTables::bpb) and K2 runs its 16-entry LookupVector / findNode instantiation; every field is
compared bit-exactly with the oracle and with the golden vectors (oracle output re-derived by
tests/refmodel.py before it was written, tests/golden/make_golden.py --large)."""
from __future__ import annotations

from pathlib import Path

import numpy as np
import pytest

from oversim_amd import KbrEngine, KbrError, Params, workload as W
from oracle_lib import OracleNet, kad_params
from test_gpu_kad_tables import _explicit_tables

pytestmark = pytest.mark.gpu
GOLD = Path(__file__).resolve().parent / "golden"
FIELDS = ("responsible", "hops", "status", "one_way_hops", "latency_ns")
LARGE = dict(k=16, lookupRedundantNodes=16, s=8)


def _eq(a, b, label, rpcs=True, hops=True):
    for f in FIELDS + (("rpcs",) if rpcs else ()):
        x, y = np.asarray(a[f]).astype(np.int64), np.asarray(b[f]).astype(np.int64)
        bad = np.nonzero(x != y)[0]
        assert len(bad) == 0, f"{label}: {f} differs at {bad[:8]}: gpu={x[bad[:8]]} ref={y[bad[:8]]}"
    if hops:
        H = b["hop_seq"].shape[1]
        assert np.array_equal(a["hop_seq"][:, :H], b["hop_seq"]), f"{label}: hop sequences"


@pytest.mark.parametrize("name", ["kad_n1000_large", "kad_n1000_large_a3"])
def test_golden_vectors(engine: KbrEngine, name):
    g = np.load(GOLD / f"{name}.npz")
    engine.set_params(Params.kademlia().replace(k=int(g["k"]), s=int(g["s"]), lookupRedundantNodes=int(g["redundant"]),
                                                lookupParallelRpcs=int(g["alpha"]),
                                                simtimeRound=int(g["simtime_round"]), kadSeed=int(g["kad_seed"])))
    engine.kad_load(g["ids"], g["xy"])
    R = int(g["redundant"])
    nodes, cnt, sib = engine.findNode(g["fn_node"], g["fn_key"], R, 1, max_out=16)
    assert np.array_equal(nodes[:, :g["fn_out"].shape[1]], g["fn_out"])
    assert np.array_equal(sib, g["fn_sib"])
    r = engine.lookup(g["keys"], g["src"], record_hops=True, count_rpcs=True)
    _eq(r, {f: g[f] for f in FIELDS + ("rpcs", "hop_seq")}, name)


def test_tables_match_oracle(engine: KbrEngine):
    net = W.population(3000, 0x16)
    engine.set_params(Params.kademlia().replace(**LARGE))
    engine.kad_load(net.ids, net.xy)
    sib, cnt, nodes = engine.kad_tables()
    osib, ocnt, onodes = OracleNet("kademlia", net.ids, net.xy, kad_params(**LARGE)).kad_tables()
    assert np.array_equal(cnt, ocnt) and cnt.max() == 16
    assert np.array_equal(nodes, onodes)
    for v in range(0, net.n, 7):
        assert set(sib[v][sib[v] != 0xFFFFFFFF]) == set(osib[v][osib[v] != 0xFFFFFFFF])


@pytest.mark.parametrize("alpha,k,r,n", [(1, 16, 16, 1000), (3, 16, 16, 1000), (1, 16, 16, 1 << 16),
                                         (3, 16, 8, 1 << 16), (2, 12, 12, 20000), (4, 16, 16, 20000)])
def test_route_matches_oracle(engine: KbrEngine, alpha, k, r, n):
    net = W.population(n, 0x1600 + alpha + k + n % 97)
    kw = dict(k=k, lookupRedundantNodes=r, s=8, lookupParallelRpcs=alpha)
    engine.set_params(Params.kademlia().replace(**kw))
    engine.kad_load(net.ids, net.xy)
    o = OracleNet("kademlia", net.ids, net.xy, kad_params(**kw), lazy=n > 100_000)
    k1, s1 = W.lookups(net.ids, 4000, 61 + alpha, node_ids=True)
    k2, s2 = W.lookups(net.ids, 4000, 71 + alpha, node_ids=False)
    keys, src = np.concatenate([k1, k2]), np.concatenate([s1, s2])
    g = engine.lookup(keys, src, record_hops=True, count_rpcs=True)
    ref = o.route(keys, src, record_hops=True, count_rpcs=True)
    _eq(g, ref, f"k={k} R={r} alpha={alpha} n={n}", hops=False)
    assert np.array_equal(g["hop_seq"], ref["hop_seq"])


@pytest.mark.parametrize("ns", [-1, 3, 0])
def test_lookup_calls_match_oracle(engine: KbrEngine, ns):
    net = W.population(1000, 0x1617)
    engine.set_params(Params.kademlia().replace(**LARGE))
    engine.kad_load(net.ids, net.xy)
    o = OracleNet("kademlia", net.ids, net.xy, kad_params(**LARGE))
    keys, src = W.lookups(net.ids, 3000, 81, node_ids=True)
    g = engine.lookupCall(keys, src, ns)
    r = o.lookup_call(keys, src, ns)
    for f in ("num_siblings", "hops", "status", "is_valid", "latency_ns", "siblings"):
        assert np.array_equal(np.asarray(g[f]).astype(np.int64), np.asarray(r[f]).astype(np.int64)), f


def test_find_node_batch_matches_oracle(engine: KbrEngine):
    net = W.population(5000, 0x1618)
    engine.set_params(Params.kademlia().replace(**LARGE))
    engine.kad_load(net.ids, net.xy)
    o = OracleNet("kademlia", net.ids, net.xy, kad_params(**LARGE))
    rng = np.random.default_rng(3)
    node = rng.integers(0, net.n, 2000).astype(np.uint32)
    keys = np.concatenate([W.random_keys(1000, rng), net.ids[rng.integers(0, net.n, 1000)]])
    for nr, ns in ((16, 1), (16, 8), (5, 1)):
        got, cnt, sib = engine.findNode(node, keys, nr, ns, max_out=16)
        for i in range(len(node)):
            ref, flag = o.find_node(int(node[i]), keys[i], nr, ns)
            assert list(got[i, :cnt[i]]) == [int(x) for x in ref], (nr, ns, i)
            assert bool(sib[i]) == flag, (nr, ns, i)


@pytest.mark.parametrize("alpha", [1, 3])
def test_explicit_tables_k16(engine: KbrEngine, alpha):
    """Non-converged k = 16 tables through ovs_kad_load_tables (partial, shuffled buckets, short
    sibling tables)."""
    net, t = _explicit_tables(2000, 1601, k=16, s=8)
    kw = dict(LARGE, lookupParallelRpcs=alpha)
    engine.set_params(Params.kademlia().replace(**kw))
    engine.kad_load_tables(net.ids, net.xy, t["siblings"], t["bucket_count"], t["bucket_nodes"])
    sib, cnt, nodes = engine.kad_tables()
    assert np.array_equal(cnt, t["bucket_count"]) and np.array_equal(nodes, t["bucket_nodes"])
    o = OracleNet("kademlia", net.ids, net.xy, kad_params(**kw), tables=t)
    k1, s1 = W.lookups(net.ids, 3000, 91 + alpha, node_ids=True)
    k2, s2 = W.lookups(net.ids, 3000, 95 + alpha, node_ids=False)
    keys, src = np.concatenate([k1, k2]), np.concatenate([s1, s2])
    g = engine.lookup(keys, src, record_hops=True, count_rpcs=True)
    r = o.route(keys, src, record_hops=True, count_rpcs=True)
    _eq(g, r, f"explicit k=16 alpha={alpha}", hops=False)
    assert np.array_equal(g["hop_seq"], r["hop_seq"])


def test_refresh_k16(engine: KbrEngine):
    """Bucket refresh with bucketRefreshNodes = k = 16 and the sibling refresh (5s = 40)."""
    net = W.population(2000, 0x1619)
    kw = dict(LARGE, lookupParallelRpcs=3)
    engine.set_params(Params.kademlia().replace(**kw))
    engine.kad_load(net.ids, net.xy)
    o = OracleNet("kademlia", net.ids, net.xy, kad_params(**kw))
    nodes = np.arange(3, net.n, 37, dtype=np.uint32)
    keys, src = o.refresh_keys(nodes)
    k1, s1 = engine.kad_refresh_keys(nodes)
    assert np.array_equal(k1, keys) and np.array_equal(s1, src)
    for R, K, S in ((16, keys, src), (40, net.ids[nodes], nodes), (8, keys[::2], src[::2])):
        r = engine.kad_refresh(K, S, R)
        e = o.exhaustive(K, S, R)
        for f in ("num_siblings", "hops", "status", "is_valid", "latency_ns", "rpcs"):
            assert np.array_equal(r[f], e[f]), (R, f)
        assert np.array_equal(r["siblings"][:, :R], e["siblings"]), R
        assert np.array_equal(r["responders"], e["responders"]) and np.array_equal(r["rtt_ns"], e["rtt_ns"]), R


@pytest.mark.parametrize("world,alpha,ns", [(2, 3, None), (4, 1, None), (4, 3, 8), (3, 3, 0)])
def test_sharded_k16_matches_single_context(engine: KbrEngine, world, alpha, ns):
    """KademliaLarge on W arcs (W contexts on one GPU, the in-process exchange): findNode answers of
    up to 16 nodes travel as ovs_kad_resp16 records; every lookup (one-way or LookupCall) equals the
    single-context K2's."""
    import torch
    from oversim_amd.shard import KadShardStepper, arc_bounds, done_to_numpy, route_kad_local_shards
    n, m = 6000, 1500
    net = W.population(n, 0x16A + world)
    bounds = arc_bounds(n, world)
    dev = torch.device("cuda", 0)
    params = Params.kademlia().replace(lookupParallelRpcs=alpha, **LARGE)
    ks, ss, qb, allk, alls = [], [], [], [], []
    for r in range(world):
        k, s0 = W.lookups(net.ids, m, 0x170 + r, node_ids=(r % 2 == 0))
        s0 = (bounds[r] + s0.astype(np.int64) % (bounds[r + 1] - bounds[r])).astype(np.uint32)
        ks.append(torch.from_numpy(k.view(np.int32)).to(dev))
        ss.append(torch.from_numpy(s0.view(np.int32)).to(dev))
        qb.append(r * m)
        allk.append(k); alls.append(s0)
    allk, alls = np.concatenate(allk), np.concatenate(alls)
    steppers = [KadShardStepper(net.ids, net.xy, bounds, r, dev, params=params, lookup_siblings=ns)
                for r in range(world)]
    assert all(st.resp_bytes == 200 for st in steppers)
    dones, rounds = route_kad_local_shards(steppers, ks, ss, qb)
    assert rounds >= 2
    engine.set_params(params)
    engine.kad_load(net.ids, net.xy)
    if ns is None:
        d = np.concatenate([done_to_numpy(x) for x in dones])
        d = d[np.argsort(d["qid"])]
        assert np.array_equal(d["qid"], np.arange(world * m))
        ref = engine.lookup(allk, alls, count_rpcs=True)
        for f in ("responsible", "hops", "status", "one_way_hops", "latency_ns"):
            assert np.array_equal(d[f].astype(np.int64), ref[f].astype(np.int64)), f
        assert np.array_equal(d["pad"].astype(np.int64), ref["rpcs"].astype(np.int64))
    else:
        ref = engine.lookupCall(allk, alls, ns)
        for r in range(world):
            qid, lo, sib = steppers[r].lookup_results(dones[r])
            for f in ("num_siblings", "hops", "status", "is_valid", "latency_ns"):
                assert np.array_equal(lo[f].astype(np.int64), np.asarray(ref[f])[qid].astype(np.int64)), (r, f)
            nsl = max(ns, 1)
            assert np.array_equal(sib[:, :nsl], np.asarray(ref["siblings"])[qid][:, :nsl])


def test_shard_refuses_capacity_change_mid_batch():
    """the shard buffers are sized for the findNode capacity fixed at begin (8 here);
    moving lookupRedundantNodes across 8 between begin and step must be refused (OVS_ESTATE) by
    step, serve and deliver, not run a 16-wide layout in 8-wide buffers."""
    import torch
    from oversim_amd.shard import KadShardStepper, arc_bounds
    n, m = 3000, 256
    net = W.population(n, 0x16F)
    bounds = arc_bounds(n, 2)
    dev = torch.device("cuda", 0)
    st = KadShardStepper(net.ids, net.xy, bounds, 0, dev, params=Params.kademlia())
    k, s0 = W.lookups(net.ids, m, 0x171, node_ids=True)
    s0 = (s0.astype(np.int64) % bounds[1]).astype(np.uint32)
    st.begin(torch.from_numpy(k.view(np.int32)).to(dev), torch.from_numpy(s0.view(np.int32)).to(dev), 0)
    st.eng.set_params(Params.kademlia().replace(lookupRedundantNodes=16))
    with pytest.raises(KbrError, match="capacity"):
        st.step()
    req = torch.zeros((4, 32), dtype=torch.uint8, device=dev)
    with pytest.raises(KbrError, match="capacity"):
        st.serve(req)
    with pytest.raises(KbrError, match="capacity"):
        st.deliver(torch.zeros((4, 104), dtype=torch.uint8, device=dev))
    # back to the begin-time capacity: the batch runs
    st.eng.set_params(Params.kademlia())
    st.step()
    torch.cuda.synchronize()
