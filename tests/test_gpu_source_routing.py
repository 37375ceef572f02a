"""source-routing-recursive on the GPU through the drop-in boundary (ovs_route_batch /
ovs_lookup_batch with routingType 4): Chord converged rings take K1's recursive path, Kademlia
takes k_kad_recursive with the visited-hop check (MODE 4) and LookupCall responses along the
reversed route (MODE 5, oversim_amd/csrc/kad_general.hip) -- against the committed golden vectors
and, on non-converged explicit tables where the visited check changes routes, against the oracle."""
from __future__ import annotations

from pathlib import Path

import numpy as np
import pytest

from oracle_lib import OracleNet, kad_params
from oversim_amd import KbrEngine, Params, workload as W
from test_source_routing import harsh_tables

pytestmark = pytest.mark.gpu
GOLD = Path(__file__).resolve().parent / "golden"


def test_chord_source_routing_matches_golden(engine: KbrEngine):
    g = np.load(GOLD / "srcroute_n2000.npz")
    rnd = int(g["simtime_round"])
    engine.set_params(Params.chord().replace(routingType=4, simtimeRound=rnd))
    engine.chord_load(g["chord_ids"], g["chord_xy"])
    r = engine.lookup(g["chord_keys"], g["chord_src"], record_hops=True)
    for f in ("responsible", "hops", "status", "one_way_hops", "latency_ns"):
        assert np.array_equal(r[f].astype(np.int64), g[f"chord_{f}"].astype(np.int64)), ("chord", f)
    assert np.array_equal(r["hop_seq"][:, :g["chord_hop_seq"].shape[1]], g["chord_hop_seq"])


def test_kad_source_routing_matches_golden(engine: KbrEngine):
    g = np.load(GOLD / "srcroute_n2000.npz")
    rnd = int(g["simtime_round"])
    engine.set_params(Params.kademlia().replace(routingType=4, simtimeRound=rnd))
    engine.kad_load(g["kad_ids"], g["kad_xy"])
    for record in (True, False):
        r = engine.lookup(g["kad_keys"], g["kad_src"], record_hops=record)
        for f in ("responsible", "hops", "status", "one_way_hops", "latency_ns"):
            assert np.array_equal(r[f].astype(np.int64), g[f"kad_{f}"].astype(np.int64)), ("kademlia", record, f)
        if record:
            assert np.array_equal(r["hop_seq"][:, :g["kad_hop_seq"].shape[1]], g["kad_hop_seq"])
    for ns in (1, 8, 0):
        lc = engine.lookupCall(g["kad_keys"], g["kad_src"], ns)
        for f in ("num_siblings", "status", "is_valid", "latency_ns", "siblings"):
            assert np.array_equal(np.asarray(lc[f]).astype(np.int64), g[f"kad_lc_ns{ns}_{f}"].astype(np.int64)), (ns, f)
        assert (np.asarray(lc["hops"]) == 0).all()


@pytest.mark.parametrize("b", [1, 2])
def test_source_routing_matches_oracle_on_explicit_tables(engine: KbrEngine, b):
    net, t = harsh_tables(1500, 0x5c70 + b, b)
    p = dict(b=b, routingType=4, hopCountMax=12)
    engine.set_params(Params.kademlia().replace(**p))
    engine.kad_load_tables_csr(net.ids, net.xy, t["siblings"], t["bucket_off"], t["bucket_nodes"])
    o = OracleNet("kademlia", net.ids, net.xy, kad_params(**p), tables=t)
    k1, s1 = W.lookups(net.ids, 20000, 19, node_ids=True)
    k2, s2 = W.lookups(net.ids, 20000, 20, node_ids=False)
    keys, src = np.concatenate([k1, k2]), np.concatenate([s1, s2])
    g = engine.lookup(keys, src, record_hops=True)
    r = o.route(keys, src, record_hops=True)
    for f in ("responsible", "hops", "status", "one_way_hops", "latency_ns"):
        assert np.array_equal(g[f].astype(np.int64), r[f].astype(np.int64)), (b, f)
    assert np.array_equal(g["hop_seq"], r["hop_seq"])
    semi = OracleNet("kademlia", net.ids, net.xy, kad_params(**{**p, "routingType": 1}), tables=t).route(keys, src)
    assert (semi["latency_ns"] != r["latency_ns"]).any()     # the visited-hop check changed some routes
    for ns in (1, 3, 0):
        lg = engine.lookupCall(keys, src, ns)
        lo = o.lookup_call(keys, src, ns)
        for f in ("num_siblings", "hops", "status", "is_valid", "latency_ns", "siblings"):
            assert np.array_equal(np.asarray(lg[f]).astype(np.int64), np.asarray(lo[f]).astype(np.int64)), (b, ns, f)
