"""R/Kademlia on the GPU (k_kad_recursive, oversim_amd/csrc/kad_general.hip): semi- and
full-recursive one-way routes and recursive LookupCalls (RecursiveLookup.cc:52-139; the hook of
Kademlia.cc:1022-1057 costs every forwarding hop a KademliaRoutingInfoMessage ahead of the route
message) through the drop-in boundary, against the committed golden vectors (snapshot tables)
and against the oracle on non-converged explicit tables (k-stride and CSR, b = 2)."""
from __future__ import annotations

from pathlib import Path

import numpy as np
import pytest

from oracle_lib import OracleNet, kad_params
from oversim_amd import KbrEngine, Params, workload as W
from test_kad_recursive import _perturbed_tables

pytestmark = pytest.mark.gpu
GOLD = Path(__file__).resolve().parent / "golden"
NONE = 0xFFFFFFFF


@pytest.mark.parametrize("name", ["kad_n2000_rec", "kad_n1000_rec_hcm3"])
@pytest.mark.parametrize("rt", [1, 2])
def test_recursive_matches_golden(engine: KbrEngine, name, rt):
    g = np.load(GOLD / f"{name}.npz")
    engine.set_params(Params.kademlia().replace(routingType=rt, simtimeRound=int(g["simtime_round"]),
                                                hopCountMax=int(g["hop_count_max"])))
    engine.kad_load(g["ids"], g["xy"])
    r = engine.lookup(g["keys"], g["src"], record_hops=True, count_rpcs=True)
    for f in ("responsible", "hops", "status", "one_way_hops", "latency_ns"):
        assert np.array_equal(r[f].astype(np.int64), g[f].astype(np.int64)), (name, rt, f)
    assert np.array_equal(r["hop_seq"][:, :g["hop_seq"].shape[1]], g["hop_seq"])
    assert (r["rpcs"] == 0).all()
    for ns in (1, 8, 0):
        lc = engine.lookupCall(g["keys"], g["src"], ns)
        for f in ("num_siblings", "status", "is_valid", "latency_ns", "siblings"):
            assert np.array_equal(np.asarray(lc[f]).astype(np.int64), g[f"lc{rt}_ns{ns}_{f}"].astype(np.int64)), \
                (name, rt, ns, f)
        assert (np.asarray(lc["hops"]) == 0).all()        # RecursiveLookup::getMinHops() = 0


@pytest.mark.parametrize("b", [1, 2])
@pytest.mark.parametrize("rt", [1, 2])
def test_recursive_matches_oracle_on_explicit_tables(engine: KbrEngine, b, rt):
    net, t = _perturbed_tables(1500, 0x4b70 + b, b)
    p = dict(b=b, routingType=rt, hopCountMax=12)
    engine.set_params(Params.kademlia().replace(**p))
    engine.kad_load_tables_csr(net.ids, net.xy, t["siblings"], t["bucket_off"], t["bucket_nodes"])
    o = OracleNet("kademlia", net.ids, net.xy, kad_params(**p), tables=t)
    k1, s1 = W.lookups(net.ids, 1500, 9, node_ids=True)
    k2, s2 = W.lookups(net.ids, 1500, 10, node_ids=False)
    keys, src = np.concatenate([k1, k2]), np.concatenate([s1, s2])
    g = engine.lookup(keys, src, record_hops=True)
    r = o.route(keys, src, record_hops=True)
    for f in ("responsible", "hops", "status", "one_way_hops", "latency_ns"):
        assert np.array_equal(g[f].astype(np.int64), r[f].astype(np.int64)), (b, rt, f)
    assert np.array_equal(g["hop_seq"], r["hop_seq"])
    for ns in (1, 3, 0):
        lg = engine.lookupCall(keys, src, ns)
        lo = o.lookup_call(keys, src, ns)
        for f in ("num_siblings", "hops", "status", "is_valid", "latency_ns", "siblings"):
            assert np.array_equal(np.asarray(lg[f]).astype(np.int64), np.asarray(lo[f]).astype(np.int64)), (b, rt, ns, f)


def test_recursive_k_stride_tables(engine: KbrEngine):
    """The same through ovs_kad_load_tables (K2's 160-bucket rows)."""
    net, t = _perturbed_tables(1500, 0x4b72, 1)
    o0 = OracleNet("kademlia", net.ids, net.xy, kad_params(), tables=t)
    sib, cnt, nodes = o0.kad_tables()
    p = dict(routingType=2, hopCountMax=12)
    engine.set_params(Params.kademlia().replace(**p))
    engine.kad_load_tables(net.ids, net.xy, sib, cnt, nodes)
    o = OracleNet("kademlia", net.ids, net.xy, kad_params(**p), tables=dict(siblings=sib, bucket_count=cnt,
                                                                             bucket_nodes=nodes))
    keys, src = W.lookups(net.ids, 3000, 11, node_ids=False)
    g = engine.lookup(keys, src)
    r = o.route(keys, src)
    for f in ("responsible", "hops", "status", "latency_ns"):
        assert np.array_equal(g[f].astype(np.int64), r[f].astype(np.int64)), f
    lg, lo = engine.lookupCall(keys, src, 8), o.lookup_call(keys, src, 8)
    for f in ("num_siblings", "status", "is_valid", "latency_ns", "siblings"):
        assert np.array_equal(np.asarray(lg[f]).astype(np.int64), np.asarray(lo[f]).astype(np.int64)), f
