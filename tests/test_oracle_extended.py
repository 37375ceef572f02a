"""Chord extendedFingerTable in the oracle (CPU; test infrastructure only).

Reference: Chord.cc:416-419 (getMaxNumRedundantNodes = numFingerCandidates), 627-641
(closestPreceedingNode asks getFinger(i, key)), 1228-1287 (a finger entry holds its FixfingersResponse:
the finger and its first numFingerCandidates successors); ChordFingerTable.cc:195-228 (getFinger(pos,
key) keeps the candidates that do not reach past the key); IterativeLookup.cc:157-244 (the start asks
the source's findNode for getMaxNumRedundantNodes() nodes) and 840-846 (lookupMerge = false: a
response replaces nextHops).

What the rules imply, checked here: the first start candidate is the non-extended choice and every
later FindNodeCall asks for one node, so routes, hop counts and latencies equal the non-extended
table's unless a first FindNodeCall times out -- then the extended lookup tries the next candidate.
"""
from __future__ import annotations

import numpy as np
import pytest

import oracle_lib as O
from oversim_amd import workload as W

FIELDS = ("responsible", "hops", "status", "latency_ns")


def _route(net, p, k, s, lazy=False):
    return O.OracleNet("chord", net.ids, net.xy, p, lazy=lazy).route(k, s, record_hops=True)


@pytest.mark.parametrize("n,seed,node_ids,sls", [(2, 4, True, 8), (3, 5, False, 8), (5, 6, True, 2), (17, 1, True, 8),
                                                 (300, 2, False, 8), (300, 7, True, 3), (2500, 3, True, 8)])
def test_extended_equals_plain_without_timeouts(n, seed, node_ids, sls):
    """rpcUdpTimeout 1.5 s against at most ~0.4 s of RTT on the 150 x 150 field: no call times out.
    Tiny rings (a finger's candidate list stops at the asking node) and numFingerCandidates above the
    successor list size (the FixfingersResponse carries min(sls, nfc) successors) included."""
    net = W.population(n, seed)
    k, s = W.lookups(net.ids, 1500, seed + 7, node_ids=node_ids)
    a = _route(net, O.chord_params(successorListSize=sls), k, s)
    for nfc in (1, 3, 8, 12):
        b = _route(net, O.chord_params(successorListSize=sls, extendedFingerTable=1, numFingerCandidates=nfc), k, s)
        for f in FIELDS:
            assert np.array_equal(a[f], b[f]), (n, nfc, f)
        assert np.array_equal(a["hop_seq"], b["hop_seq"]), (n, nfc)


def test_extended_recursive_and_lookup_calls_equal_plain():
    net = W.population(1200, 5)
    k, s = W.lookups(net.ids, 800, 11, node_ids=False)
    for rt in (1, 2):
        a = _route(net, O.chord_params(routingType=rt), k, s)
        b = _route(net, O.chord_params(routingType=rt, extendedFingerTable=1), k, s)
        for f in FIELDS:
            assert np.array_equal(a[f], b[f]), (rt, f)
    a = O.OracleNet("chord", net.ids, net.xy).lookup_call(k, s)
    b = O.OracleNet("chord", net.ids, net.xy, O.chord_params(extendedFingerTable=1)).lookup_call(k, s)
    for f in ("num_siblings", "hops", "status", "is_valid", "latency_ns"):
        assert np.array_equal(a[f], b[f]), f
    assert np.array_equal(a["siblings"], b["siblings"])


def test_extended_retries_the_next_candidate_after_a_first_timeout():
    """rpcUdpTimeout 0.25 s: many first calls time out.  The plain table then fails the lookup; the
    extended one sends to the next start candidate at the timeout, so more lookups succeed, and a
    lookup whose first call answered is unchanged."""
    net = W.population(2500, 3)
    k, s = W.lookups(net.ids, 2000, 10, node_ids=True)
    a = _route(net, O.chord_params(rpcUdpTimeout=0.25), k, s)
    b = _route(net, O.chord_params(rpcUdpTimeout=0.25, extendedFingerTable=1), k, s)
    lazy = _route(net, O.chord_params(rpcUdpTimeout=0.25, extendedFingerTable=1), k, s, lazy=True)
    for f in FIELDS:
        assert np.array_equal(b[f], lazy[f]), f          # stored and lazily evaluated rings agree
    ok_a, ok_b = a["status"] == 0, b["status"] == 0
    assert ok_b.sum() > ok_a.sum()
    assert not np.any(ok_a & ~ok_b)                      # a retry never loses a lookup
    same = ok_a & ok_b
    for f in FIELDS:
        assert np.array_equal(a[f][same], b[f][same]), f
    # the rescued lookups paid the timeout before their first answered call
    rescued = ~ok_a & ok_b
    assert rescued.any()
    assert np.all(b["latency_ns"][rescued] >= 250_000_000)


def test_extended_refused_on_explicit_tables():
    """Explicit tables hold one node per finger, not the FixfingersResponse candidate lists."""
    n = 200
    net = W.population(n, 6)
    fingers = O.OracleNet("chord", net.ids, net.xy).chord_fingers()
    tables = dict(pred=((np.arange(n) - 1) % n).astype(np.uint32),
                  succ=((np.arange(n)[:, None] + 1 + np.arange(8)[None, :]) % n).astype(np.uint32),
                  nsucc=np.full(n, 8, np.uint8), fingers=fingers, deque_size=np.full(n, 160, np.uint8))
    O.OracleNet("chord", net.ids, net.xy, tables=tables)         # accepted without the extended table
    with pytest.raises(RuntimeError, match="extendedFingerTable"):
        O.OracleNet("chord", net.ids, net.xy, O.chord_params(extendedFingerTable=1), tables=tables)


# ---- a second reading of the extended findNode, straight from the reference's code paths ----------
M160 = 1 << 160


def _between(x, a, b, lo_closed, hi_closed):
    """OverlayKey::isBetween / R / L / LR (OverlayKey.cc:587-644), literally."""
    if not lo_closed and not hi_closed:
        if x == a:
            return False
        return a < x < b if a < b else (x > a or x < b)
    if a == b and x == a:
        return True
    lo = (lambda: x >= a) if lo_closed else (lambda: x > a)
    hi = (lambda: x <= b) if hi_closed else (lambda: x < b)
    return (lo() and hi()) if a <= b else (lo() or hi())


def _find_node_ext(ids, node, key, nfc, sls):
    """Chord::findNode(key, nfc, 1) with extendedFingerTable on the stable ring (Chord.cc:548-599,
    600-674; ChordFingerTable.cc:195-228; the finger entries as handleRpcFixfingersResponse stores
    them, 1268-1287)."""
    n = len(ids)
    ns = min(sls, n - 1)
    me = ids[node]
    succ = [(node + 1 + j) % n for j in range(ns)]
    pred = ids[(node - 1) % n]
    if _between(key, pred, me, False, True):                  # isSiblingFor(thisNode, key, 1)
        return [node]
    if _between(key, me, ids[succ[0]], False, True):           # key in (me, succ0]
        return succ[:nfc]
    temp = None
    for s in reversed(succ):                                   # closestPreceedingNode 604-611
        if _between(ids[s], me, key, False, True):
            temp = s
            break
    d0 = (ids[succ[0]] - me) % M160
    for i in range(159, -1, -1):
        trivial = (1 << i) <= d0
        if trivial:
            f = succ[0]
        else:
            lk = (me + (1 << i)) % M160
            f = next((j for j in range(n) if ids[j] >= lk), 0)   # responsible(me + 2^i)
        if _between(ids[f], ids[temp], key, True, True):
            if trivial:
                return [succ[0]]
            out = []
            for j in range(-1, min(min(sls, n - 1), nfc)):
                c = f if j < 0 else (f + 1 + j) % n
                if c == node:
                    break
                if not _between(key, ids[f], ids[c], True, True):
                    out.append(c)
            return (out or [f])[:nfc]
    out = []
    for s in reversed(succ):
        if len(out) > nfc:
            break
        if _between(ids[s], me, key, False, False):
            out.append(s)
    return out[:nfc]


@pytest.mark.parametrize("n,seed,sls", [(3, 11, 8), (40, 12, 4), (500, 13, 8)])
def test_extended_find_node_matches_second_reading(n, seed, sls):
    from oversim_amd.kbr import key_to_int
    net = W.population(n, seed)
    ids = [key_to_int(net.ids[i]) for i in range(n)]
    rng = np.random.default_rng(seed)
    for nfc in (1, 3, 6):
        o = O.OracleNet("chord", net.ids, net.xy, O.chord_params(successorListSize=sls, extendedFingerTable=1,
                                                                numFingerCandidates=nfc))
        keys, _ = W.lookups(net.ids, 120, seed + nfc, node_ids=False)
        nodes = rng.integers(0, n, len(keys))
        for i in range(len(keys)):
            got, _ = o.find_node(int(nodes[i]), keys[i], nfc, 1)
            assert got == _find_node_ext(ids, int(nodes[i]), key_to_int(keys[i]), nfc, sls), (n, nfc, i)
