"""R/Kademlia on the CPU: recursive one-way routes and recursive LookupCalls (semi- and
full-recursive) over Kademlia tables -- BaseOverlay::sendToKey / handleBaseOverlayMessage
(BaseOverlay.cc:880-1004, 1380-1582), Kademlia::recursiveRoutingHook (Kademlia.cc:1022-1057),
RecursiveLookup (RecursiveLookup.cc:52-139), the route-RPC response paths (BaseOverlay.cc:
1779-1822).  The oracle reproduces its committed golden vectors (tests/golden/kad_*_rec*.npz,
made by make_golden.py --kadrec after refmodel.KadRecursiveSim agreed), and agrees with the
refmodel on non-converged and b = 2 tables."""
from __future__ import annotations

from pathlib import Path

import numpy as np
import pytest

import refmodel
from oracle_lib import OracleNet, kad_params
from oversim_amd import workload as W

GOLD = Path(__file__).resolve().parent / "golden"
NONE = 0xFFFFFFFF


@pytest.mark.parametrize("name", ["kad_n2000_rec", "kad_n1000_rec_hcm3"])
def test_oracle_reproduces_recursive_kad_golden(name):
    g = np.load(GOLD / f"{name}.npz")
    rnd, hcm = int(g["simtime_round"]), int(g["hop_count_max"])
    for rt in (1, 2):
        o = OracleNet("kademlia", g["ids"], g["xy"], kad_params(routingType=rt, simtimeRound=rnd, hopCountMax=hcm))
        if rt == 1:
            r = o.route(g["keys"], g["src"], record_hops=True)
            for f in ("responsible", "hops", "status", "one_way_hops", "latency_ns"):
                assert np.array_equal(r[f], g[f]), (name, f)
            assert np.array_equal(r["hop_seq"][:, :g["hop_seq"].shape[1]], g["hop_seq"])
        for ns in (1, 8, 0):
            lc = o.lookup_call(g["keys"], g["src"], ns)
            for f in ("num_siblings", "status", "is_valid", "latency_ns", "siblings"):
                assert np.array_equal(np.asarray(lc[f]), g[f"lc{rt}_ns{ns}_{f}"]), (name, rt, ns, f)
    # the R/Kademlia hook costs every forwarding hop a KademliaRoutingInfoMessage ahead of the route
    # message: semi- and full-recursive LookupCalls differ only in the way back
    ok = (g["lc1_ns8_is_valid"] == 1) & (g["lc2_ns8_is_valid"] == 1)
    assert ok.mean() > 0.9
    assert (g["lc2_ns8_latency_ns"][ok] != g["lc1_ns8_latency_ns"][ok]).mean() > 0.5


def _perturbed_tables(n, seed, b=1):
    """Non-converged CSR tables: bucket members dropped (30 %), buckets shuffled, some sibling tables cut."""
    net = W.population(n, seed)
    p = kad_params(b=b)
    sib, off, nodes = OracleNet("kademlia", net.ids, net.xy, p).kad_tables_csr()
    rng = np.random.default_rng(seed)
    new_off, out = np.zeros_like(off), []
    for j in range(len(off) - 1):
        seg = [int(x) for x in nodes[off[j]:off[j + 1]] if rng.random() > 0.3]
        rng.shuffle(seg)
        out += seg
        new_off[j + 1] = len(out)
    sib = sib.copy()
    for v in range(n):
        row = [int(x) for x in sib[v] if x != NONE]
        if rng.random() < 0.2:
            row = row[:int(rng.integers(2, len(row)))]
        sib[v, :] = NONE
        sib[v, :len(row)] = row
    return net, dict(siblings=sib, bucket_off=new_off, bucket_nodes=np.array(out, dtype=np.uint32))


@pytest.mark.parametrize("b", [1, 2])
@pytest.mark.parametrize("rt", [1, 2])
def test_recursive_matches_refmodel_on_explicit_tables(b, rt):
    net, t = _perturbed_tables(600, 0x4b60 + b, b)
    p = kad_params(b=b, routingType=rt, hopCountMax=12)
    o = OracleNet("kademlia", net.ids, net.xy, p, tables=t)
    nb = refmodel.kad_num_buckets(b)
    buckets = []
    for v in range(net.n):
        row = {}
        for m in range(nb):
            a, z = int(t["bucket_off"][v * nb + m]), int(t["bucket_off"][v * nb + m + 1])
            if z > a:
                row[m] = [int(x) for x in t["bucket_nodes"][a:z]]
        buckets.append(row)
    sibsorted = o.kad_tables_csr()[0]           # the oracle keeps sibling tables XOR-sorted
    T = refmodel.KadTables(net.ids, sibsorted, None, None, k=p.k, s=p.s, b=b, buckets=buckets)
    sim = refmodel.KadRecursiveSim(T, net.xy, hop_max=12)
    k1, s1 = W.lookups(net.ids, 300, 7, node_ids=True)
    k2, s2 = W.lookups(net.ids, 300, 8, node_ids=False)
    keys, src = np.concatenate([k1, k2]), np.concatenate([s1, s2])
    r = o.route(keys, src, record_hops=True)
    for i in range(len(keys)):
        m = sim.route(keys[i], int(src[i]))
        for f in ("responsible", "hops", "status", "latency_ns"):
            assert int(r[f][i]) == int(m[f]), (b, rt, i, f)
    statuses = set()
    for ns in (1, 3, 0):
        lc = o.lookup_call(keys, src, ns)
        for i in range(len(keys)):
            m = sim.lookup_call(keys[i], int(src[i]), ns, full=(rt == 2))
            for f in ("num_siblings", "status", "is_valid", "latency_ns"):
                assert int(lc[f][i]) == int(m[f]), (b, rt, ns, i, f)
            assert [int(x) for x in lc["siblings"][i] if x != NONE] == m["siblings"][:max(ns, 1)]
        statuses |= set(int(x) for x in lc["status"])
    assert 0 in statuses and 6 in statuses     # answered, and answered without the siblings flag
