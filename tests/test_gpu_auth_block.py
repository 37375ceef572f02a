"""measureAuthBlock = true on the GPU (ABI 12) against the oracle and the committed golden vectors.

BaseOverlay.ned's measureAuthBlock (default.ini:399) makes every RPC response carry
AUTHBLOCK_L = SIGNATURE_L + CERT_L + PUBKEY_L = 800 bits (CommonMessages.msg:45-47, 57, 73):
each FindNodeResponse / LookupResponse is 100 B longer, which moves every RTT and so every
latency, and through rpcUdpTimeout / LOOKUP_TIMEOUT can change routes.  Calls and the one-way
route message keep their size.  Same bar as every other path: bit-exact fields, int64-ns latency.
"""
from __future__ import annotations

from pathlib import Path

import numpy as np
import pytest

from oversim_amd import KbrEngine, Params, workload as W
from oracle_lib import OracleNet, chord_params, kad_params

pytestmark = pytest.mark.gpu
GOLD = Path(__file__).resolve().parent / "golden"
ROUTE = ("responsible", "hops", "status", "one_way_hops", "latency_ns")
LOOKUP = ("num_siblings", "hops", "status", "is_valid", "latency_ns")


def _eq(a, b, fields, label):
    for f in fields:
        x, y = np.asarray(a[f]).astype(np.int64), np.asarray(b[f]).astype(np.int64)
        bad = np.nonzero(x != y)[0]
        assert len(bad) == 0, f"{label}: {f} differs at {bad[:8]}: gpu={x[bad[:8]]} ref={y[bad[:8]]}"


def test_chord_golden(engine: KbrEngine):
    g = np.load(GOLD / "chord_n1000_auth.npz")
    assert int(g["measure_auth_block"]) == 1
    engine.set_params(Params.chord().replace(measureAuthBlock=1, simtimeRound=int(g["simtime_round"])))
    engine.chord_load(g["ids"], g["xy"])
    r = engine.lookup(g["keys"], g["src"], record_hops=True)
    _eq(r, g, ROUTE, "chord_n1000_auth")
    H = g["hop_seq"].shape[1]
    assert np.array_equal(r["hop_seq"][:, :H], g["hop_seq"])


def test_kad_golden(engine: KbrEngine):
    g = np.load(GOLD / "kad_n2000_a3_auth.npz")
    engine.set_params(Params.kademlia().replace(measureAuthBlock=1, lookupParallelRpcs=int(g["alpha"]),
                                                simtimeRound=int(g["simtime_round"]), kadSeed=int(g["kad_seed"])))
    engine.kad_load(g["ids"], g["xy"])
    r = engine.lookup(g["keys"], g["src"], record_hops=True, count_rpcs=True)
    _eq(r, g, ROUTE + ("rpcs",), "kad_n2000_a3_auth")
    H = g["hop_seq"].shape[1]
    assert np.array_equal(r["hop_seq"][:, :H], g["hop_seq"])


def test_chord_config_c_shape(engine: KbrEngine):
    """2^20-node ring (config C's network), 200k random keys; plus the LookupCall variant."""
    net = W.population(1 << 20, 0xA17)
    engine.set_params(Params.chord().replace(measureAuthBlock=1))
    engine.chord_load(net.ids, net.xy)
    o = OracleNet("chord", net.ids, net.xy, chord_params(measureAuthBlock=1))
    keys, src = W.lookups(net.ids, 200_000, 0xA18, node_ids=False)
    r = engine.lookup(keys, src)
    _eq(r, o.route(keys, src, record_hops=False), ROUTE, "chord 2^20 auth")
    plain = OracleNet("chord", net.ids, net.xy).route(keys[:5000], src[:5000], record_hops=False)
    assert (r["latency_ns"][:5000] > plain["latency_ns"]).all()
    lc = engine.lookupCall(keys[:20000], src[:20000], 8)
    _eq(lc, o.lookup_call(keys[:20000], src[:20000], 8), LOOKUP, "chord LookupCall auth")


@pytest.mark.parametrize("alpha,rt", [(1, 0), (3, 0), (3, 1)])
def test_kad_routes_and_lookup_calls(engine: KbrEngine, alpha, rt):
    """15 000 nodes (nodes_2d_15000 coordinates): one-way routes, LookupCalls, and R/Kademlia
    semi-recursive LookupCalls, whose LookupResponse carries the auth block too."""
    net = W.population(15000, 0x4b41)
    kw = dict(measureAuthBlock=1, lookupParallelRpcs=alpha, routingType=rt)
    engine.set_params(Params.kademlia().replace(**kw))
    engine.kad_load(net.ids, net.xy)
    o = OracleNet("kademlia", net.ids, net.xy, kad_params(**kw))
    keys, src = W.lookups(net.ids, 20000, 0xA19, node_ids=True)
    if rt == 0:
        _eq(engine.lookup(keys, src, count_rpcs=True), o.route(keys, src, record_hops=False, count_rpcs=True),
            ROUTE + ("rpcs",), f"kad a{alpha} auth")
    _eq(engine.lookupCall(keys, src, 8), o.lookup_call(keys, src, 8), LOOKUP, f"kad LookupCall a{alpha} rt{rt} auth")


def test_kad_refresh_rtts(engine: KbrEngine):
    """Exhaustive-iterative refresh lookups (K2x): responder RTTs include the auth block."""
    net = W.population(2000, 0x5EF)
    kw = dict(measureAuthBlock=1, lookupParallelRpcs=3)
    engine.set_params(Params.kademlia().replace(**kw))
    engine.kad_load(net.ids, net.xy)
    o = OracleNet("kademlia", net.ids, net.xy, kad_params(**kw))
    nodes = np.arange(3, len(net.ids), 37, dtype=np.uint32)
    keys, src = o.refresh_keys(nodes)
    r, e = engine.kad_refresh(keys, src, 8), o.exhaustive(keys, src, 8)
    _eq(r, e, LOOKUP + ("rpcs",), "refresh auth")
    assert np.array_equal(r["responders"], e["responders"]) and np.array_equal(r["rtt_ns"], e["rtt_ns"])
