"""The two independent restatements of the Kademlia iterative lookup agree.

oracle/ovs_oracle.c runs each lookup as a per-lookup event list that evaluates the responder's
findNode when the call is sent; tests/refmodel.py (KadLookupSim) simulates every message hop
through an OMNeT++-style future event set and evaluates findNode when the call arrives, on its
own findNode / isSiblingFor (KadTables).  Both follow IterativeLookup.cc:133-349, 406-449,
488-689, 786-1195; parameter variations push the alpha > 1 rules the round-1 golden vectors
rested on a single reading of: accepts(step), late siblings, strictParallelRpcs, numNewRpcs,
RPC timeouts / dead nodes, LOOKUP_TIMEOUT, same-instant tx serialisation.  CPU only.
"""
from __future__ import annotations

import numpy as np
import pytest

import refmodel
from oversim_amd import workload as W
from oracle_lib import OracleNet, kad_params

FIELDS = ("responsible", "hops", "status", "one_way_hops", "latency_ns", "rpcs")

VARIANTS = {
    "a1": dict(lookupParallelRpcs=1),
    "a2": dict(lookupParallelRpcs=2),
    "a3": dict(lookupParallelRpcs=3),
    "a4_r4": dict(lookupParallelRpcs=4, lookupRedundantNodes=4),
    "a3_useall": dict(lookupParallelRpcs=3, lookupUseAllParallelResponses=1),
    "a3_nolate": dict(lookupParallelRpcs=3, lookupAcceptLateSiblings=0),
    "a3_loose": dict(lookupParallelRpcs=3, lookupStrictParallelRpcs=0),
    "a3_newresp": dict(lookupParallelRpcs=3, lookupNewRpcOnEveryResponse=1),
    # RPC timeouts fire (RTTs up to ~1.3 s on these coordinates): dead nodes, handleTimeout
    "a3_rpcto": dict(lookupParallelRpcs=3, rpcUdpTimeout=0.35),
    "a3_rpcto_newto": dict(lookupParallelRpcs=3, rpcUdpTimeout=0.35, lookupNewRpcOnEveryTimeout=1),
    "a2_lookupto": dict(lookupParallelRpcs=2, lookupTimeout=0.9),
    "a3_hcm3": dict(lookupParallelRpcs=3, hopCountMax=3),
    "a3_first": dict(lookupParallelRpcs=3, lookupFinishOnFirstUnchanged=1),
    "a3_trunc": dict(lookupParallelRpcs=3, simtimeRound=0),
    # the fork's own Kademlia configuration: lookupParallelRpcs = lookupRedundantNodes = 8
    # (maidsafe.ini:18-19), and one alpha between 4 and 8
    "a8_maidsafe": dict(lookupParallelRpcs=8, lookupRedundantNodes=8),
    "a5": dict(lookupParallelRpcs=5),
    "a8_rpcto": dict(lookupParallelRpcs=8, rpcUdpTimeout=0.35),
}


def _sim(o: OracleNet, net, p) -> refmodel.KadLookupSim:
    sib, cnt, nodes = o.kad_tables()
    tab = refmodel.KadTables(net.ids, sib, cnt, nodes, k=p.k, s=p.s)
    return refmodel.KadLookupSim(
        tab, net.xy, redundant=p.lookupRedundantNodes, alpha=p.lookupParallelRpcs, merge=bool(p.lookupMerge),
        strict=bool(p.lookupStrictParallelRpcs), visit_once=bool(p.lookupVisitOnlyOnce),
        accept_late_siblings=bool(p.lookupAcceptLateSiblings), use_all=bool(p.lookupUseAllParallelResponses),
        new_on_timeout=bool(p.lookupNewRpcOnEveryTimeout), new_on_response=bool(p.lookupNewRpcOnEveryResponse),
        finish_on_first_unchanged=bool(p.lookupFinishOnFirstUnchanged), hop_max=p.hopCountMax,
        rnd=bool(p.simtimeRound), rpc_timeout=p.rpcUdpTimeout, lookup_timeout=p.lookupTimeout, k=p.k)


@pytest.fixture(scope="module")
def net():
    return W.population(1500, 0x4b42)


@pytest.mark.parametrize("name", list(VARIANTS))
def test_one_way_lookups_agree(net, name):
    p = kad_params(**VARIANTS[name])
    o = OracleNet("kademlia", net.ids, net.xy, p)
    sim = _sim(o, net, p)
    k1, s1 = W.lookups(net.ids, 200, 11, node_ids=True)
    k2, s2 = W.lookups(net.ids, 200, 12, node_ids=False)
    keys, src = np.concatenate([k1, k2]), np.concatenate([s1, s2])
    r = o.route(keys, src, record_hops=True, count_rpcs=True)
    statuses = set()
    for i in range(len(keys)):
        m = sim.run(keys[i], int(src[i]))
        for f in FIELDS:
            assert int(r[f][i]) == int(m[f]), (name, i, f, int(r[f][i]), int(m[f]))
        assert [int(x) for x in r["hop_seq"][i] if x != 0xFFFFFFFF] == m["hop_seq"], (name, i)
        statuses.add(int(m["status"]))
    if "rpcto" in name or "lookupto" in name or "hcm" in name:
        assert statuses != {0}, f"{name}: the variant should exercise a failure path"


@pytest.mark.parametrize("alpha,ns", [(1, 8), (3, 8), (3, 3)])
def test_lookup_calls_agree(net, alpha, ns):
    """KBRTestApp LookupCalls (numSiblings > 1): sibling vectors, hops, validity, duration."""
    p = kad_params(lookupParallelRpcs=alpha)
    o = OracleNet("kademlia", net.ids, net.xy, p)
    sim = _sim(o, net, p)
    keys, src = W.lookups(net.ids, 300, 13 + alpha, node_ids=(ns == 8))
    r = o.lookup_call(keys, src, ns)
    for i in range(len(keys)):
        m = sim.run(keys[i], int(src[i]), num_siblings=ns, lookup_call=True)
        assert int(r["is_valid"][i]) == m["is_valid"], i
        assert int(r["hops"][i]) == m["hops"], i
        assert int(r["latency_ns"][i]) == m["latency_ns"], i
        assert int(r["num_siblings"][i]) == len(m["siblings"]), i
        assert [int(x) for x in r["siblings"][i][: len(m["siblings"])]] == m["siblings"], i


REFRESH_VARIANTS = {
    "a3": dict(lookupParallelRpcs=3),
    "a1": dict(lookupParallelRpcs=1),
    "a3_loose": dict(lookupParallelRpcs=3, lookupStrictParallelRpcs=0),
    # RPC timeouts: dead nodes leave nextHops (IterativeLookup.cc:948-957), evicted nodes re-enter
    "a3_rpcto": dict(lookupParallelRpcs=3, rpcUdpTimeout=0.35),
    "a3_rpcto_newto": dict(lookupParallelRpcs=3, rpcUdpTimeout=0.35, lookupNewRpcOnEveryTimeout=1),
    "a2_lookupto": dict(lookupParallelRpcs=2, lookupTimeout=0.9),
    "a3_hcm12": dict(lookupParallelRpcs=3, hopCountMax=12),
    "a8": dict(lookupParallelRpcs=8),
}


@pytest.mark.parametrize("name", list(REFRESH_VARIANTS))
@pytest.mark.parametrize("R", [8, 40])
def test_refresh_lookups_agree(net, name, R):
    """Exhaustive-iterative refresh lookups (Kademlia.cc:1591-1686): the bucket refresh keys
    (R = bucketRefreshNodes = 8) and the sibling refresh of the node's own key (R = 5s = 40)."""
    p = kad_params(**REFRESH_VARIANTS[name])
    o = OracleNet("kademlia", net.ids, net.xy, p)
    sim = _sim(o, net, p)
    nodes = np.arange(7, len(net.ids), 149, dtype=np.uint32)
    if R == 8:
        keys, src = o.refresh_keys(nodes)
        keys, src = keys[::3], src[::3]
    else:
        keys, src = net.ids[nodes], nodes
    r = o.exhaustive(keys, src, R)
    statuses, lost = set(), False
    for i in range(len(keys)):
        m = sim.run(keys[i], int(src[i]), num_siblings=R, lookup_call=True, exhaustive=R)
        assert int(r["is_valid"][i]) == m["is_valid"], (name, i)
        assert int(r["status"][i]) == m["status"], (name, i)
        assert int(r["hops"][i]) == m["hops"], (name, i)
        assert int(r["rpcs"][i]) == m["rpcs"], (name, i)
        assert int(r["latency_ns"][i]) == m["latency_ns"], (name, i)
        assert int(r["num_siblings"][i]) == len(m["siblings"]), (name, i)
        assert [int(x) for x in r["siblings"][i][: len(m["siblings"])]] == m["siblings"], (name, i)
        H = len(m["responders"])
        assert [int(x) for x in r["responders"][i][:H]] == m["responders"], (name, i)
        assert [int(x) for x in r["rtt_ns"][i][:H]] == m["rtt_ns"], (name, i)
        statuses.add(int(m["status"]))
        lost |= m["rpcs"] > len(m["responders"])
    if "rpcto" in name:   # exhaustive lookups succeed through dead nodes: timeouts show as lost calls
        assert lost, f"{name}: the variant should time some FindNodeCalls out"
    elif "to" in name or "hcm" in name:
        assert statuses != {0}, f"{name}: the variant should exercise a failure path"


def test_refresh_keys_follow_the_timer(net):
    """handleBucketRefreshTimerExpired's keys: self ^ 2^i for i = 159 .. msb(self ^ closest
    sibling), filtered by the stale mask."""
    o = OracleNet("kademlia", net.ids, net.xy, kad_params())
    sib, _, _ = o.kad_tables()
    ids = [refmodel.to_int(w) for w in net.ids]
    nodes = np.array([0, 5, 700, len(ids) - 1], dtype=np.uint32)
    keys, src = o.refresh_keys(nodes)
    exp = []
    for v in nodes:
        front = min(ids[x] ^ ids[v] for x in sib[v] if x != 0xFFFFFFFF)
        for i in range(159, front.bit_length() - 2, -1):
            exp.append((int(v), ids[v] ^ (1 << i)))
    assert [(int(s), refmodel.to_int(k)) for k, s in zip(keys, src)] == exp
    stale = np.zeros((len(nodes), 5), dtype=np.uint32)
    stale[:, 4] = 0x80000000            # only bucket 159
    keys2, src2 = o.refresh_keys(nodes, stale)
    assert list(src2) == list(nodes)
    assert [refmodel.to_int(k) for k in keys2] == [ids[v] ^ (1 << 159) for v in nodes]


@pytest.mark.parametrize("alpha", [1, 3])
def test_exhaustive_routing_type_agrees(net, alpha):
    """routingType = "exhaustive-iterative" (BaseOverlay.cc:1434-1442): one-way lookups (numSiblings 1,
    the route message to the closest node found) and LookupCalls (numSiblings = s)."""
    p = kad_params(lookupParallelRpcs=alpha, routingType=3)
    o = OracleNet("kademlia", net.ids, net.xy, p)
    sim = _sim(o, net, p)
    keys, src = W.lookups(net.ids, 150, 41 + alpha, node_ids=False)
    r = o.route(keys, src, record_hops=True, count_rpcs=True)
    for i in range(len(keys)):
        m = sim.run(keys[i], int(src[i]), exhaustive=8)
        for f in FIELDS:
            assert int(r[f][i]) == int(m[f]), (alpha, i, f, int(r[f][i]), int(m[f]))
        assert [int(x) for x in r["hop_seq"][i] if x != 0xFFFFFFFF] == m["hop_seq"], (alpha, i)
    c = o.lookup_call(keys, src, 8)
    for i in range(len(keys)):
        m = sim.run(keys[i], int(src[i]), num_siblings=8, lookup_call=True, exhaustive=8)
        assert int(c["is_valid"][i]) == m["is_valid"] and int(c["hops"][i]) == m["hops"], i
        assert int(c["latency_ns"][i]) == m["latency_ns"], i
        assert [int(x) for x in c["siblings"][i][: len(m["siblings"])]] == m["siblings"], i


@pytest.mark.parametrize("alpha", [1, 3])
def test_exact_key_lookup_calls_agree(net, alpha):
    """LookupCalls with numSiblings = 0 (IterativeLookup.cc:149, 171-184, 313, 862-870): the lookup
    ends at the first response carrying the key's node; keys no node holds fail."""
    p = kad_params(lookupParallelRpcs=alpha)
    o = OracleNet("kademlia", net.ids, net.xy, p)
    sim = _sim(o, net, p)
    k1, s1 = W.lookups(net.ids, 150, 51 + alpha, node_ids=True)
    k2, s2 = W.lookups(net.ids, 50, 61 + alpha, node_ids=False)
    keys, src = np.concatenate([k1, k2, net.ids[:5]]), np.concatenate([s1, s2, np.arange(5, dtype=np.uint32)])
    r = o.lookup_call(keys, src, 0)
    valid = 0
    for i in range(len(keys)):
        m = sim.run(keys[i], int(src[i]), num_siblings=0, lookup_call=True)
        assert int(r["is_valid"][i]) == m["is_valid"], i
        assert int(r["status"][i]) == m["status"], i
        assert int(r["hops"][i]) == m["hops"], i
        assert int(r["latency_ns"][i]) == m["latency_ns"], i
        assert [int(x) for x in r["siblings"][i][: len(m["siblings"])]] == m["siblings"], i
        valid += m["is_valid"]
    assert 150 <= valid < len(keys)      # node-ID keys and own keys found, random keys not


# [Config KademliaLarge] (omnetpp.ini:113-126): k = 16, lookupRedundantNodes = 16, s = 8, alpha = 1
LARGE_VARIANTS = {
    "large_a1": dict(k=16, lookupRedundantNodes=16, lookupParallelRpcs=1),
    "large_a3": dict(k=16, lookupRedundantNodes=16, lookupParallelRpcs=3),
    "k16_r8_a3": dict(k=16, lookupRedundantNodes=8, lookupParallelRpcs=3),
    "k12_r12_a2": dict(k=12, lookupRedundantNodes=12, lookupParallelRpcs=2),
}


@pytest.mark.parametrize("name", list(LARGE_VARIANTS))
def test_kademlia_large_lookups_agree(net, name):
    """16-entry buckets and LookupVectors: the two readings agree on one-way lookups and LookupCalls."""
    p = kad_params(**LARGE_VARIANTS[name])
    o = OracleNet("kademlia", net.ids, net.xy, p)
    sim = _sim(o, net, p)
    k1, s1 = W.lookups(net.ids, 150, 21, node_ids=True)
    k2, s2 = W.lookups(net.ids, 150, 22, node_ids=False)
    keys, src = np.concatenate([k1, k2]), np.concatenate([s1, s2])
    r = o.route(keys, src, record_hops=True, count_rpcs=True)
    for i in range(len(keys)):
        m = sim.run(keys[i], int(src[i]))
        for f in FIELDS:
            assert int(r[f][i]) == int(m[f]), (name, i, f, int(r[f][i]), int(m[f]))
        assert [int(x) for x in r["hop_seq"][i] if x != 0xFFFFFFFF] == m["hop_seq"], (name, i)
    lc = o.lookup_call(k1, s1, 8)
    for i in range(len(k1)):
        m = sim.run(k1[i], int(s1[i]), num_siblings=8, lookup_call=True)
        assert int(lc["is_valid"][i]) == m["is_valid"] and int(lc["hops"][i]) == m["hops"], (name, i)
        assert int(lc["latency_ns"][i]) == m["latency_ns"], (name, i)
        assert [int(x) for x in lc["siblings"][i][: len(m["siblings"])]] == m["siblings"], (name, i)


def test_kademlia_large_refresh_agrees(net):
    """Bucket refresh with bucketRefreshNodes = k = 16 (exhaustive-iterative, R = 16)."""
    p = kad_params(k=16, lookupRedundantNodes=16, lookupParallelRpcs=3)
    o = OracleNet("kademlia", net.ids, net.xy, p)
    sim = _sim(o, net, p)
    nodes = np.arange(3, len(net.ids), 211, dtype=np.uint32)
    keys, src = o.refresh_keys(nodes)
    keys, src = keys[::4], src[::4]
    r = o.exhaustive(keys, src, 16)
    for i in range(len(keys)):
        m = sim.run(keys[i], int(src[i]), num_siblings=16, lookup_call=True, exhaustive=16)
        assert int(r["status"][i]) == m["status"] and int(r["hops"][i]) == m["hops"], i
        assert int(r["rpcs"][i]) == m["rpcs"] and int(r["latency_ns"][i]) == m["latency_ns"], i
        assert [int(x) for x in r["siblings"][i][: len(m["siblings"])]] == m["siblings"], i
