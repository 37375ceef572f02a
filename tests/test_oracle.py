"""CPU tests of the oracle itself (no GPU).

1. OverlayKey known answers: the input cases of OverlayKey::test()
   (OverlayKey.cc:720-828) with answers derived by hand from the documented
   semantics (the reference prints them for eyeballing; it stores no expected
   values except the SHA-1 lines, which are off this path).
2. Randomised OverlayKey operations against Python big-int arithmetic mod 2^160.
3. Oracle vs the independent Python restatement (refmodel) and the committed
   golden vectors.
"""
from __future__ import annotations

from pathlib import Path

import numpy as np
import pytest

import oracle_lib as O
import refmodel
from oversim_amd import key_from_int, workload as W

M = 1 << 160
MAX = M - 1
GOLD = Path(__file__).resolve().parent / "golden"


def K(x):
    return key_from_int(x)


def between(which, x, a, b, unspec=0):
    return bool(O.lib().orc_key_between(which, O._p(K(x)), O._p(K(a)), O._p(K(b)), unspec))


def test_overlaykey_test_cases():
    L = O.lib()
    cmp = lambda a, b: L.orc_key_cmp(O._p(K(a)), O._p(K(b)))  # noqa: E731
    assert cmp(256, 10) > 0 and not cmp(256, 10) < 0            # "256 < 10 = 0", "256 > 10 = 1"
    assert between(0, 10, 3, 256) is True                      # 10 isBetween(3, 256)
    assert between(0, 3, 10, 256) is False                     # 3 isBetween(10, 256)
    assert between(0, 256, 10, 256) is False                   # 256 isBetween(10, 256): open
    assert between(1, 256, 10, 256) is True                    # 256 isBetweenR(10, 256)
    assert between(0, MAX, MAX - 1, 0) is True                 # max isBetween(max-1, 0)
    assert between(0, MAX - 1, MAX, 1) is False                # max-1 isBetween(max, 1)
    assert between(2, MAX - 1, MAX - 1, 1) is True             # max-1 isBetweenL(max-1, 1)
    assert between(2, 1, MAX - 1, 1) is False                  # 1 isBetweenL(max-1, 1)
    assert between(1, 1, MAX - 1, 1) is True                   # 1 isBetweenR(max-1, 1)
    assert between(0, 1, MAX - 1, 1) is False                  # 1 isBetween(max-1, 1)
    assert between(0, 1, MAX - 1, 0) is False                  # 1 isBetween(max-1, 0)
    # the reference adds a full 64-bit limb for the equal top limb although only 32 of its
    # bits are significant (OverlayKey.cc:540-551): 64 + 64 + 55 = 183, not 151
    assert L.orc_key_shared_prefix(O._p(K(256)), O._p(K(3)), 1) == 183
    assert L.orc_key_shared_prefix(O._p(K(256)), O._p(K(256)), 1) == 160
    out = np.zeros(5, np.uint32)
    L.orc_key_add(O._p(K(MAX)), O._p(K(1)), O._p(out))
    assert refmodel.to_int(out) == 0                           # wrap-around: max + 1 = 0
    L.orc_key_add(O._p(K(MAX)), O._p(K(2)), O._p(out))
    assert refmodel.to_int(out) == 1
    L.orc_key_sub(O._p(K(0)), O._p(K(1)), O._p(out))
    assert refmodel.to_int(out) == MAX
    L.orc_key_sub(O._p(K(0)), O._p(K(2)), O._p(out))
    assert refmodel.to_int(out) == MAX - 1
    assert cmp(MAX, 1) > 0
    # KeyUniRingMetric::distance(1, max) = max - 1; (max, 1) = 2 (Comparator.h:137-153)
    L.orc_key_sub(O._p(K(MAX)), O._p(K(1)), O._p(out))
    assert refmodel.to_int(out) == MAX - 1
    L.orc_key_sub(O._p(K(1)), O._p(K(MAX)), O._p(out))
    assert refmodel.to_int(out) == 2
    for i in range(160):                                       # pow2 / log2 test
        L.orc_key_pow2(i, O._p(out))
        assert refmodel.to_int(out) == 1 << i
        assert L.orc_key_log2(O._p(out)) == i
    assert L.orc_key_log2(O._p(K(0))) == -1


def test_equal_endpoint_rules():
    a = 12345
    assert between(0, a, a, a) is False            # (a, a): x == a excluded
    assert between(0, a + 1, a, a) is True         # (a, a) = whole ring minus a
    assert between(1, a, a, a) is True             # (a, a]: a == b && x == a
    assert between(1, a + 1, a, a) is False
    assert between(2, a, a, a) is True
    assert between(3, a, a, a) is True
    for which in range(4):
        for m in (1, 2, 4):                        # any unspecified operand -> false
            assert between(which, 5, 1, 10, unspec=m) is False


def test_key_ops_match_bigint():
    rng = np.random.default_rng(1)
    L = O.lib()
    out = np.zeros(5, np.uint32)
    for _ in range(3000):
        a, b, x = (int(rng.integers(0, 1 << 62)) << 98 ^ int(rng.integers(0, 1 << 62)) << 30 ^ int(rng.integers(0, 1 << 30))
                   for _ in range(3))
        a, b, x = a % M, b % M, x % M
        if rng.random() < 0.2:
            b = a
        if rng.random() < 0.2:
            x = a
        L.orc_key_add(O._p(K(a)), O._p(K(b)), O._p(out))
        assert refmodel.to_int(out) == (a + b) % M
        L.orc_key_sub(O._p(K(a)), O._p(K(b)), O._p(out))
        assert refmodel.to_int(out) == (a - b) % M
        L.orc_key_xor(O._p(K(a)), O._p(K(b)), O._p(out))
        assert refmodel.to_int(out) == a ^ b
        c = L.orc_key_cmp(O._p(K(a)), O._p(K(b)))
        assert (c > 0) == (a > b) and (c == 0) == (a == b)
        assert between(0, x, a, b) == refmodel.between(x, a, b)
        assert between(1, x, a, b) == refmodel.between_r(x, a, b)
        assert between(3, x, a, b) == refmodel.between_lr(x, a, b)
        spl = L.orc_key_shared_prefix(O._p(K(a)), O._p(K(b)), 1)
        bl = (a ^ b).bit_length()
        assert spl == (160 if a == b else (160 - bl if bl > 128 else 192 - bl))   # same top-limb quirk
        p, n = int(rng.integers(0, 129)), int(rng.integers(1, 33))
        assert L.orc_key_bit_range(O._p(K(a)), p, n) == (a >> p) & ((1 << n) - 1)


def _auth(g) -> int:
    return int(g["measure_auth_block"]) if "measure_auth_block" in g.files else 0


@pytest.mark.parametrize("name", ["chord_n1000_round", "chord_n1000_trunc", "chord_n9", "chord_n2", "chord_n1000_auth"])
def test_oracle_reproduces_chord_golden(name):
    g = np.load(GOLD / f"{name}.npz")
    o = O.OracleNet("chord", g["ids"], g["xy"], O.chord_params(simtimeRound=int(g["simtime_round"]),
                                                               measureAuthBlock=_auth(g)))
    r = o.route(g["keys"], g["src"], record_hops=True)
    for f in ("responsible", "hops", "status", "one_way_hops", "latency_ns"):
        assert np.array_equal(r[f], g[f]), f
    assert np.array_equal(r["hop_seq"][:, :g["hop_seq"].shape[1]], g["hop_seq"])


@pytest.mark.parametrize("name", ["kad_n2000_a1", "kad_n2000_a3", "kad_n2000_a3_auth"])
def test_oracle_reproduces_kad_golden(name):
    g = np.load(GOLD / f"{name}.npz")
    p = O.kad_params(lookupParallelRpcs=int(g["alpha"]), simtimeRound=int(g["simtime_round"]), kadSeed=int(g["kad_seed"]),
                     measureAuthBlock=_auth(g))
    o = O.OracleNet("kademlia", g["ids"], g["xy"], p)
    r = o.route(g["keys"], g["src"], record_hops=True, count_rpcs=True)
    for f in ("responsible", "hops", "status", "one_way_hops", "latency_ns", "rpcs"):
        assert np.array_equal(r[f], g[f]), f


def test_oracle_matches_refmodel_chord_random_rings():
    for n, seed in ((17, 1), (300, 2), (2500, 3)):
        net = W.population(n, seed)
        k, s = W.lookups(net.ids, 400, seed + 7, node_ids=bool(seed % 2))
        r = O.OracleNet("chord", net.ids, net.xy).route(k, s, record_hops=True)
        ring = refmodel.ChordRing(net.ids, net.xy)
        for i in range(len(k)):
            m = ring.lookup(k[i], int(s[i]))
            for f in ("responsible", "hops", "status", "latency_ns"):
                assert int(r[f][i]) == int(m[f]), (n, i, f)


def test_oracle_kademlia_findnode_matches_refmodel():
    net = W.population(1200, 9)
    o = O.OracleNet("kademlia", net.ids, net.xy)
    sib, cnt, nodes = o.kad_tables()
    tab = refmodel.KadTables(net.ids, sib, cnt, nodes)
    rng = np.random.default_rng(3)
    for i in range(300):
        c = int(rng.integers(0, 1200))
        key = W.random_keys(1, rng)[0] if i % 2 else net.ids[int(rng.integers(0, 1200))]
        res, flag = o.find_node(c, key, 8, 1)
        assert [int(x) for x in res] == tab.find_node(c, refmodel.to_int(key), 8, 1)
        assert flag == tab.is_sibling_for(c, refmodel.to_int(key), 1)


def test_kademlia_sibling_table_is_xor_closest():
    net = W.population(500, 11)
    o = O.OracleNet("kademlia", net.ids, net.xy)
    sib, _, _ = o.kad_tables()
    ids = [refmodel.to_int(w) for w in net.ids]
    for c in range(0, 500, 37):
        d = sorted((ids[x] ^ ids[c], x) for x in range(500) if x != c)
        assert [x for _, x in d[:40]] == [int(x) for x in sib[c]]


def test_oracle_semi_recursive_matches_refmodel():
    """Recursive one-way routing (ChordLarge: routingType = semi-recursive): the oracle's
    full sendToKey restatement (recNumRedundantNodes = 3, loop detection) equals the
    greedy forwarding walk of the independent model on converged rings."""
    for n, seed, hcm in ((17, 1, 50), (300, 2, 50), (2500, 3, 50), (2500, 4, 3)):
        net = W.population(n, seed)
        k, s = W.lookups(net.ids, 400, seed + 7, node_ids=bool(seed % 2))
        p = O.chord_params(routingType=1, hopCountMax=hcm)
        r = O.OracleNet("chord", net.ids, net.xy, p).route(k, s, record_hops=True, count_rpcs=True)
        assert not r["rpcs"].any()
        ring = refmodel.ChordRing(net.ids, net.xy)
        for i in range(len(k)):
            m = ring.lookup_recursive(k[i], int(s[i]), hop_max=hcm)
            for f in ("responsible", "hops", "status", "one_way_hops", "latency_ns"):
                assert int(r[f][i]) == int(m[f]), (n, i, f)
            if m["status"] == 0:
                assert list(r["hop_seq"][i][:m["hops"]]) == m["hop_seq"]


def test_semi_recursive_path_is_iterative_path():
    """On a converged ring both modes visit the same nodes; only the accounting differs:
    recursive hop count = iterative responders (+0), latency = sum of per-hop route messages."""
    net = W.population(3000, 5)
    k, s = W.lookups(net.ids, 500, 6)
    it = O.OracleNet("chord", net.ids, net.xy).route(k, s, record_hops=True)
    rc = O.OracleNet("chord", net.ids, net.xy, O.chord_params(routingType=1)).route(k, s, record_hops=True)
    ok = (it["status"] == 0) & (rc["status"] == 0)
    assert ok.mean() > 0.99
    assert np.array_equal(it["responsible"][ok], rc["responsible"][ok])
    assert np.array_equal(it["hops"][ok], rc["hops"][ok])
    assert np.array_equal(it["hop_seq"][ok], rc["hop_seq"][ok])


@pytest.mark.parametrize("name", ["chord_n1000_semirec", "chord_n1000_semirec_hcm4"])
def test_oracle_reproduces_recursive_golden(name):
    g = np.load(GOLD / f"{name}.npz")
    p = O.chord_params(simtimeRound=int(g["simtime_round"]), routingType=int(g["routing_type"]),
                       hopCountMax=int(g["hop_count_max"]))
    r = O.OracleNet("chord", g["ids"], g["xy"], p).route(g["keys"], g["src"], record_hops=True)
    for f in ("responsible", "hops", "status", "one_way_hops", "latency_ns"):
        assert np.array_equal(r[f], g[f]), f
    assert np.array_equal(r["hop_seq"][:, :g["hop_seq"].shape[1]], g["hop_seq"])


def test_oracle_fix_fingers_round_converges():
    """The oracle's synchronous fixfingers round (Chord.cc:845-875, 1228-1270) repairs a ring
    whose successor pointers are right into the converged finger table."""
    n = 800
    net = W.population(n, 71)
    ideal = O.OracleNet("chord", net.ids, net.xy).chord_fingers()
    rng = np.random.default_rng(72)
    fing = ideal.copy()
    fing[rng.random(fing.shape) < 0.4] = 0xFFFFFFFF
    pred = ((np.arange(n) - 1) % n).astype(np.uint32)
    succ = ((np.arange(n)[:, None] + 1 + np.arange(8)[None, :]) % n).astype(np.uint32)
    t = dict(pred=pred, succ=succ, nsucc=np.full(n, 8, np.uint8), fingers=fing,
             deque_size=rng.integers(120, 161, n).astype(np.uint8))
    o = O.OracleNet("chord", net.ids, net.xy, tables=t)
    r = o.chord_fix_fingers()
    assert r["ok"] > 0 and r["changed"] > 0
    assert np.array_equal(o.chord_fingers(), ideal)
    r2 = o.chord_fix_fingers()
    assert r2["changed"] == 0 and r2["ok"] == r["ok"]


# ------------------------------------------------------------ LookupCall (KBRTestApp lookup test)

@pytest.mark.parametrize("ns", [8, 3, 1])
def test_oracle_lookup_call_matches_refmodel_chord(ns):
    """orc_lookup_batch (the full IterativeLookup state machine with numSiblings = ns) vs the
    refmodel's direct loop: siblings vector, hop count, status, lookup duration."""
    for n, seed in ((2, 5), (6, 6), (300, 7), (2500, 8)):
        net = W.population(n, seed)
        k, s = W.lookups(net.ids, 300, seed + 9, node_ids=bool(seed % 2))
        r = O.OracleNet("chord", net.ids, net.xy).lookup_call(k, s, ns)
        ring = refmodel.ChordRing(net.ids, net.xy)
        for i in range(len(k)):
            m = ring.lookup_call(k[i], int(s[i]), ns)
            row = [int(x) for x in r["siblings"][i] if x != 0xFFFFFFFF]
            assert row == m["siblings"], (n, i)
            assert int(r["num_siblings"][i]) == len(m["siblings"]), (n, i)
            for f in ("hops", "status", "latency_ns"):
                assert int(r[f][i]) == int(m[f]), (n, i, f)
            assert int(r["is_valid"][i]) == (m["status"] == 0)


def test_oracle_lookup_call_chord_relates_to_route():
    """Same path as the one-way route; the lookup ends at the answering response."""
    net = W.population(3000, 12)
    o = O.OracleNet("chord", net.ids, net.xy)
    k, s = W.lookups(net.ids, 2000, 13, node_ids=True)
    a = o.route(k, s)
    b = o.lookup_call(k, s, 1)
    assert np.array_equal(a["hops"], b["hops"])
    assert np.array_equal(a["responsible"], b["siblings"][:, 0])
    local = a["responsible"] == s
    assert np.all(b["latency_ns"][local] == a["latency_ns"][local])
    assert np.all(b["latency_ns"][~local] < a["latency_ns"][~local])
    c = o.lookup_call(k, s, -1)                     # getMaxNumSiblings() = successorListSize
    assert c["siblings"].shape[1] == 8 and np.all(c["num_siblings"] == 8)
    assert np.array_equal(c["siblings"], (a["responsible"][:, None] + np.arange(8)[None, :]) % 3000)
    assert np.all(c["latency_ns"][~local] > b["latency_ns"][~local])   # 7 more NodeHandles in the answer
    with pytest.raises(ValueError):
        o.lookup_call(k[:4], s[:4], 9)               # numSiblings too big!


@pytest.mark.parametrize("ns", [8, 5, 2])
def test_oracle_kademlia_sibling_findnode_matches_refmodel(ns):
    """Kademlia::isSiblingFor / findNode with numSiblings > 1 (the LookupCall's responders)."""
    net = W.population(1200, 19)
    o = O.OracleNet("kademlia", net.ids, net.xy)
    sib, cnt, nodes = o.kad_tables()
    tab = refmodel.KadTables(net.ids, sib, cnt, nodes)
    rng = np.random.default_rng(20)
    nsib = 0
    for i in range(400):
        c = int(rng.integers(0, 1200))
        if i % 3 == 0:
            key = W.random_keys(1, rng)[0]
        else:
            # keys near c: c's own id or a close node's, so that c is often a sibling
            key = net.ids[int(sib[c][int(rng.integers(0, 12))])] if i % 3 == 1 else net.ids[c]
        res, flag = o.find_node(c, key, 8, ns)
        kk = refmodel.to_int(key)
        assert flag == tab.is_sibling_for(c, kk, ns)
        assert [int(x) for x in res] == tab.find_node(c, kk, 8, ns)
        nsib += flag
    assert 50 < nsib < 400


@pytest.mark.parametrize("alpha", [1, 3])
def test_oracle_kademlia_lookup_call_properties(alpha):
    """Kademlia LookupCall (numSiblings = s): valid lookups return s distinct nodes in XOR order
    from the answering sibling's view (not always the global s closest: the answer comes from the
    responder's own tables); node-ID keys find their node first; the lookup needs no more hops
    than the one-way route (it stops at the first responder in the key's top s)."""
    net = W.population(2000, 23)
    p = O.kad_params(lookupParallelRpcs=alpha)
    o = O.OracleNet("kademlia", net.ids, net.xy, p)
    k, s = W.lookups(net.ids, 600, 24, node_ids=True)
    r = o.lookup_call(k, s)
    a = o.route(k, s)
    assert np.all(r["is_valid"] == 1) and np.all(r["num_siblings"] == 8)
    ids = [refmodel.to_int(w) for w in net.ids]
    exact = 0
    for i in range(len(k)):
        kk = refmodel.to_int(k[i])
        row = [int(x) for x in r["siblings"][i]]
        d = [ids[x] ^ kk for x in row]
        assert d == sorted(d) and len(set(row)) == 8, i
        assert ids[row[0]] == kk, i                                 # node-ID key: its node first
        exact += row == sorted(range(2000), key=lambda x: ids[x] ^ kk)[:8]
    assert exact > len(k) // 2
    assert np.all(r["hops"] <= a["hops"])


def test_auth_block_adds_100_bytes_per_response():
    """measureAuthBlock (CommonMessages.msg:45-47, 57, 73): on a 10 Mbps channel each FindNodeResponse
    serialises 2 x 80 us longer (sender and receiver access links), calls and the route message do
    not change; with alpha = 1 Chord every accepted hop is one response, so routes are unchanged and
    latency grows by exactly hops x 160 us."""
    g = np.load(GOLD / "chord_n1000_auth.npz")
    plain = O.OracleNet("chord", g["ids"], g["xy"], O.chord_params()).route(g["keys"], g["src"], record_hops=False)
    for f in ("responsible", "hops", "status", "one_way_hops"):
        assert np.array_equal(plain[f], g[f]), f
    assert np.array_equal(g["latency_ns"] - plain["latency_ns"], g["hops"].astype(np.int64) * 160_000)
    assert (g["hops"] > 0).mean() > 0.9
