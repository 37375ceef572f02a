"""GPU parity tests for the Chord hot path (K1 chord_route, findNode batch, delay).

The HIP engine (through the C ABI) is compared with the CPU oracle on the same
seeded inputs and with the committed golden vectors.  Integer outputs
(responsible node, hop count, hop sequence, status) must be bit-exact; latency
is int64 ns and must also be exact -- the 1e-9 relative tolerance of the
north star is not needed once SimTime quantisation is reproduced.
"""
from __future__ import annotations

from pathlib import Path

import numpy as np
import pytest

from oversim_amd import KbrEngine, Params, workload as W
from oracle_lib import OracleNet, chord_params

pytestmark = pytest.mark.gpu
GOLD = Path(__file__).resolve().parent / "golden"
FIELDS = ("responsible", "hops", "status", "one_way_hops", "latency_ns")


def _eq(a: dict, b: dict, label: str, hop_cols: int | None = None):
    for f in FIELDS:
        bad = np.nonzero(np.asarray(a[f]).astype(np.int64) != np.asarray(b[f]).astype(np.int64))[0]
        assert len(bad) == 0, f"{label}: {f} differs at {bad[:8]} gpu={np.asarray(a[f])[bad[:8]]} ref={np.asarray(b[f])[bad[:8]]}"
    if hop_cols is not None and "hop_seq" in a and "hop_seq" in b:
        ha, hb = a["hop_seq"][:, :hop_cols], b["hop_seq"][:, :hop_cols]
        assert np.array_equal(ha, hb), f"{label}: hop sequences differ"


@pytest.mark.parametrize("name", ["chord_n1000_round", "chord_n1000_trunc", "chord_n9", "chord_n2"])
def test_golden_vectors(engine: KbrEngine, name):
    g = np.load(GOLD / f"{name}.npz")
    engine.set_params(Params.chord().replace(simtimeRound=int(g["simtime_round"])))
    engine.chord_load(g["ids"], g["xy"])
    r = engine.lookup(g["keys"], g["src"], record_hops=True)
    H = g["hop_seq"].shape[1]
    _eq(r, {f: g[f] for f in FIELDS} | {"hop_seq": g["hop_seq"]}, name, hop_cols=H)


def test_fingers_match_oracle(engine: KbrEngine):
    net = W.population(5000, 21)
    engine.set_params(Params.chord())
    engine.chord_load(net.ids, net.xy)
    o = OracleNet("chord", net.ids, net.xy)
    assert np.array_equal(engine.chord_fingers(), o.chord_fingers())


def test_delay_matches_oracle(engine: KbrEngine):
    net = W.population(3000, 22)
    engine.set_params(Params.chord())
    engine.chord_load(net.ids, net.xy)
    o = OracleNet("chord", net.ids, net.xy)
    rng = np.random.default_rng(5)
    a = rng.integers(0, 3000, 4000).astype(np.uint32)
    b = rng.integers(0, 3000, 4000).astype(np.uint32)
    b[:50] = a[:50]   # src == dst -> 0 delay
    nb = rng.choice([83, 87, 269, 186, 61, 1500], 4000).astype(np.int32)
    gpu = engine.delay_ns(a, b, nb)
    ref = np.array([o.delay_ns(int(x), int(y), int(z)) for x, y, z in zip(a, b, nb)])
    assert np.array_equal(gpu, ref)


@pytest.mark.parametrize("nr,ns", [(1, 1), (3, 1), (8, 8), (1, 8)])
def test_find_node_matches_oracle(engine: KbrEngine, nr, ns):
    net = W.population(2000, 23)
    engine.set_params(Params.chord())
    engine.chord_load(net.ids, net.xy)
    o = OracleNet("chord", net.ids, net.xy)
    rng = np.random.default_rng(6)
    node = rng.integers(0, 2000, 3000).astype(np.uint32)
    keys = np.concatenate([W.random_keys(1500, rng), net.ids[rng.integers(0, 2000, 1500)]])
    # keys just around the node: its own id, pred, successors
    keys[:100] = net.ids[node[:100]]
    keys[100:200] = net.ids[(node[100:200].astype(np.int64) + 3) % 2000]
    nodes, cnt, sib = engine.findNode(node, keys, nr, ns)
    for i in range(len(node)):
        ref, flag = o.find_node(int(node[i]), keys[i], nr, ns)
        assert list(nodes[i, :cnt[i]]) == ref, (i, nodes[i, :cnt[i]], ref)
        assert bool(sib[i]) == flag


@pytest.mark.parametrize("rnd", [1, 0])
def test_route_medium_ring(engine: KbrEngine, rnd):
    net = W.population(1 << 16, 24)
    engine.set_params(Params.chord().replace(simtimeRound=rnd))
    engine.chord_load(net.ids, net.xy)
    o = OracleNet("chord", net.ids, net.xy, chord_params(simtimeRound=rnd))
    k1, s1 = W.lookups(net.ids, 20000, 31, node_ids=True)
    k2, s2 = W.lookups(net.ids, 20000, 32, node_ids=False)
    keys, src = np.concatenate([k1, k2]), np.concatenate([s1, s2])
    g = engine.lookup(keys, src, record_hops=True)
    r = o.route(keys, src, record_hops=True)
    _eq(g, r, f"2^16 ring rnd={rnd}", hop_cols=50)


@pytest.mark.parametrize("sls,hcm", [(1, 50), (2, 50), (3, 6), (8, 4), (5, 0), (12, 50), (16, 50)])
def test_route_successor_list_and_hop_limit(engine: KbrEngine, sls, hcm):
    """successorListSize (the window the WinRec / NodeRec distances cover; beyond its 8 entries the
    kernel scans the successors exactly) and hopCountMax variants of the converged-ring kernel
    against the oracle, node-ID and random keys."""
    net = W.population(1 << 14, 40 + sls)
    p = dict(successorListSize=sls, hopCountMax=hcm)
    engine.set_params(Params.chord().replace(**p))
    engine.chord_load(net.ids, net.xy)
    o = OracleNet("chord", net.ids, net.xy, chord_params(**p))
    k1, s1 = W.lookups(net.ids, 20000, 41 + sls, node_ids=True)
    k2, s2 = W.lookups(net.ids, 20000, 42 + sls, node_ids=False)
    keys, src = np.concatenate([k1, k2]), np.concatenate([s1, s2])
    g = engine.lookup(keys, src, record_hops=True)
    r = o.route(keys, src, record_hops=True)
    _eq(g, r, f"successorListSize={sls} hopCountMax={hcm}", hop_cols=max(hcm, 1))


def test_params_change_rebuilds_node_records(engine: KbrEngine):
    """successorListSize changed after the load: the node records are rebuilt for it."""
    net = W.population(5000, 47)
    engine.set_params(Params.chord())
    engine.chord_load(net.ids, net.xy)
    keys, src = W.lookups(net.ids, 20000, 48, node_ids=True)
    engine.lookup(keys, src)
    engine.set_params(Params.chord().replace(successorListSize=2))
    g = engine.lookup(keys, src, record_hops=True)
    r = OracleNet("chord", net.ids, net.xy, chord_params(successorListSize=2)).route(keys, src, record_hops=True)
    _eq(g, r, "successorListSize 8 -> 2", hop_cols=50)


def test_route_1m_ring_vs_oracle(engine: KbrEngine):
    """Config C ring size (2^20 nodes, random coordinates) on a 200k-lookup sample."""
    net = W.population(1 << 20, 0xC)
    engine.set_params(Params.chord())
    engine.chord_load(net.ids, net.xy)
    o = OracleNet("chord", net.ids, net.xy)
    keys, src = W.lookups(net.ids, 200_000, 33, node_ids=False)
    g = engine.lookup(keys, src, record_hops=True)
    r = o.route(keys, src, record_hops=True)
    _eq(g, r, "2^20 ring", hop_cols=50)


def test_route_large_batch_properties(engine: KbrEngine):
    """Full-size batch (config C: 10M lookups on 2^20 nodes): size-independent properties."""
    net = W.population(1 << 20, 0xC)
    engine.set_params(Params.chord())
    engine.chord_load(net.ids, net.xy)
    keys, src = W.lookups(net.ids, 10_000_000, 34, node_ids=False)
    g = engine.lookup(keys, src)
    assert np.all(g["status"] == 0)
    # the responsible node of a key is its ring successor (isSiblingFor, Chord.cc:452-457)
    top = (net.ids[:, 4].astype(np.uint64) << 32) | net.ids[:, 3].astype(np.uint64)
    ktop = (keys[:, 4].astype(np.uint64) << 32) | keys[:, 3].astype(np.uint64)
    sample = np.arange(0, len(keys), 997)
    pos = np.searchsorted(top, ktop[sample], side="left")
    exact = pos < len(top)
    exact &= top[np.minimum(pos, len(top) - 1)] != ktop[sample]   # unambiguous on the top 64 bits
    expect = np.where(pos == len(top), 0, pos)
    assert np.array_equal(g["responsible"][sample][exact], expect[exact])
    # latency lower bound: every counted hop costs at least the 4 serialisation delays
    assert np.all(g["latency_ns"] >= g["hops"].astype(np.int64) * 272000)
    assert 9.0 < g["hops"].mean() < 11.5


def test_explicit_tables_match_oracle(engine: KbrEngine):
    """ovs_chord_load_tables: non-converged snapshot (unspecified fingers, holes in the deque)."""
    n = 400
    net = W.population(n, 25)
    rng = np.random.default_rng(7)
    o_ideal = OracleNet("chord", net.ids, net.xy)
    fing = o_ideal.chord_fingers().copy()
    # knock out ~30% of finger entries and shrink some deques
    mask = rng.random(fing.shape) < 0.3
    fing[mask] = 0xFFFFFFFF
    deque = rng.integers(100, 161, n).astype(np.uint8)
    pred = ((np.arange(n) - 1) % n).astype(np.uint32)
    succ = ((np.arange(n)[:, None] + 1 + np.arange(8)[None, :]) % n).astype(np.uint32)
    nsucc = np.full(n, 8, dtype=np.uint8)
    nsucc[rng.integers(0, n, 40)] = rng.integers(1, 8, 40).astype(np.uint8)
    tables = dict(pred=pred, succ=succ, nsucc=nsucc, fingers=fing, deque_size=deque)
    o = OracleNet("chord", net.ids, net.xy, tables=tables)
    engine.set_params(Params.chord())
    engine.chord_load_tables(net.ids, net.xy, pred, succ, nsucc, fing, deque)
    assert np.array_equal(engine.chord_fingers(), o.chord_fingers())
    k1, s1 = W.lookups(net.ids, 3000, 35, node_ids=True)
    k2, s2 = W.lookups(net.ids, 3000, 36, node_ids=False)
    keys, src = np.concatenate([k1, k2]), np.concatenate([s1, s2])
    g = engine.lookup(keys, src, record_hops=True)
    r = o.route(keys, src, record_hops=True)
    _eq(g, r, "explicit tables", hop_cols=50)


def _broken_tables(n, seed):
    """A non-converged snapshot: ~30% of finger entries unspecified, deques shrunk, some short
    successor lists (correct pred/succ0)."""
    net = W.population(n, seed)
    rng = np.random.default_rng(seed + 1)
    fing = OracleNet("chord", net.ids, net.xy).chord_fingers().copy()
    fing[rng.random(fing.shape) < 0.3] = 0xFFFFFFFF
    wrong = rng.random(fing.shape) < 0.05                 # stale entries pointing anywhere
    fing[wrong] = rng.integers(0, n, int(wrong.sum())).astype(np.uint32)
    deque = rng.integers(100, 161, n).astype(np.uint8)
    pred = ((np.arange(n) - 1) % n).astype(np.uint32)
    succ = ((np.arange(n)[:, None] + 1 + np.arange(8)[None, :]) % n).astype(np.uint32)
    nsucc = np.full(n, 8, dtype=np.uint8)
    nsucc[rng.integers(0, n, n // 10)] = rng.integers(1, 8, n // 10).astype(np.uint8)
    return net, dict(pred=pred, succ=succ, nsucc=nsucc, fingers=fing, deque_size=deque)


@pytest.mark.parametrize("subset", [False, True])
def test_fix_fingers_round_matches_oracle(engine: KbrEngine, subset):
    """Batched maintenance lookups (ovs_chord_fix_fingers) vs the oracle's round: same fingers,
    same counters; a full round over a ring with correct successors reaches the ideal table."""
    n = 3000
    net, t = _broken_tables(n, 61)
    o = OracleNet("chord", net.ids, net.xy, tables=t)
    engine.set_params(Params.chord())
    engine.chord_load_tables(net.ids, net.xy, t["pred"], t["succ"], t["nsucc"], t["fingers"], t["deque_size"])
    nodes = np.arange(0, n, 3, dtype=np.uint32) if subset else None
    g = engine.chord_fix_fingers(nodes)
    r = o.chord_fix_fingers(nodes)
    assert (g["ok"], g["changed"], g["hops"]) == (r["ok"], r["changed"], r["hops"]), (g, r)
    assert g["lookups"] == g["ok"] > 0
    assert np.array_equal(engine.chord_fingers(), o.chord_fingers())
    if not subset:
        assert np.array_equal(engine.chord_fingers(), OracleNet("chord", net.ids, net.xy).chord_fingers())
    keys, src = W.lookups(net.ids, 4000, 62, node_ids=True)
    _eq(engine.lookup(keys, src, record_hops=True), o.route(keys, src, record_hops=True), "after fixfingers",
        hop_cols=50)


def test_rejects_unsupported(engine: KbrEngine):
    from oversim_amd import KbrError
    net = W.population(100, 26)
    engine.set_params(Params.chord())
    engine.chord_load(net.ids, net.xy)
    with pytest.raises(KbrError):
        engine.set_params(Params.chord().replace(jitter=0.1))
    with pytest.raises(KbrError):
        engine.chord_load(net.ids[::-1].copy(), net.xy)   # not sorted


# ------------------------------------------------------------ semi-recursive routing

@pytest.mark.parametrize("name", ["chord_n1000_semirec", "chord_n1000_semirec_hcm4"])
def test_recursive_golden_vectors(engine: KbrEngine, name):
    g = np.load(GOLD / f"{name}.npz")
    engine.set_params(Params.chord().replace(simtimeRound=int(g["simtime_round"]), routingType=1,
                                             hopCountMax=int(g["hop_count_max"])))
    engine.chord_load(g["ids"], g["xy"])
    r = engine.lookup(g["keys"], g["src"], record_hops=True, count_rpcs=True)
    _eq(r, {f: g[f] for f in FIELDS} | {"hop_seq": g["hop_seq"]}, name, hop_cols=g["hop_seq"].shape[1])
    assert not r["rpcs"].any()


@pytest.mark.parametrize("rnd,rt,hcm", [(1, 1, 50), (0, 2, 50), (1, 1, 5), (1, 1, 0)])
def test_recursive_matches_oracle(engine: KbrEngine, rnd, rt, hcm):
    net = W.population(1 << 16, 77 + rnd)
    k1, s1 = W.lookups(net.ids, 100_000, 78, node_ids=False)
    k2, s2 = W.lookups(net.ids, 100_000, 79, node_ids=True)
    keys, src = np.concatenate([k1, k2]), np.concatenate([s1, s2])
    engine.set_params(Params.chord().replace(simtimeRound=rnd, routingType=rt, hopCountMax=hcm))
    engine.chord_load(net.ids, net.xy)
    r = engine.lookup(keys, src, record_hops=True)
    o = OracleNet("chord", net.ids, net.xy, chord_params(simtimeRound=rnd, routingType=rt, hopCountMax=hcm))
    ref = o.route(keys, src, record_hops=True)
    _eq(r, ref, f"recursive rnd={rnd} hcm={hcm}", hop_cols=max(hcm, 1))
    if hcm == 0:
        assert (r["status"] == 3).all()


def test_recursive_rejects_explicit_tables(engine: KbrEngine):
    from oversim_amd import KbrError
    g = np.load(GOLD / "chord_n9.npz")
    engine.set_params(Params.chord())
    engine.chord_load(g["ids"], g["xy"])
    fingers = engine.chord_fingers()
    n = len(g["ids"])
    pred = (np.arange(n) - 1) % n
    succ = np.stack([(np.arange(n) + 1 + j) % n for j in range(8)], axis=1).astype(np.uint32)
    engine.chord_load_tables(g["ids"], g["xy"], pred, succ, np.full(n, 8, np.uint8), fingers,
                             np.full(n, 160, np.uint8))
    engine.set_params(Params.chord().replace(routingType=1))
    with pytest.raises(KbrError):
        engine.lookup(g["keys"][:4], g["src"][:4])


def test_stabilize_fixfingers_rounds_converge(engine: KbrEngine):
    """Multi-round convergence after a batch of joins: synchronous stabilize rounds
    (ovs_chord_stabilize, Chord.cc:793-842, 1055-1225) alternating with fixfingers rounds, round by
    round equal to the oracle's (the engine takes each notified node's nearest caller, the oracle
    applies the NotifyCalls one by one), ending in the stable ring; routing equal throughout."""
    from test_oracle_stabilize import joined_ring
    n = 2000
    net, joined, t = joined_ring(n, 0x57AD)
    o = OracleNet("chord", net.ids, net.xy, tables=t)
    engine.set_params(Params.chord())
    engine.chord_load_tables(net.ids, net.xy, t["pred"], t["succ"], t["nsucc"], t["fingers"], t["deque_size"])
    keys, src = W.lookups(net.ids, 3000, 0x57AE, node_ids=True)
    sub = np.arange(0, n, 2, dtype=np.uint32)
    for rnd in range(12):
        nodes = sub if rnd == 0 else None                 # a partial round first
        g, r = engine.chord_stabilize(nodes), o.chord_stabilize(nodes)
        assert (g["succ_changed"], g["lists_changed"], g["pred_changed"]) == \
            (r["succ_changed"], r["lists_changed"], r["pred_changed"]), (rnd, g, r)
        for a, b in zip(engine.chord_tables(), o.chord_lists()):
            assert np.array_equal(a, b), rnd
        gf, rf = engine.chord_fix_fingers(), o.chord_fix_fingers()
        assert (gf["ok"], gf["changed"], gf["hops"]) == (rf["ok"], rf["changed"], rf["hops"]), rnd
        assert np.array_equal(engine.chord_fingers(), o.chord_fingers()), rnd
        if rnd in (0, 2):
            _eq(engine.lookup(keys, src, record_hops=True), o.route(keys, src, record_hops=True), f"round {rnd}",
                hop_cols=50)
        if rnd > 0 and g["lists_changed"] == 0 and g["pred_changed"] == 0 and gf["changed"] == 0:
            break
    pred, succ, nsucc = engine.chord_tables()
    assert np.array_equal(pred, (np.arange(n) - 1) % n)
    assert np.array_equal(succ, (np.arange(n)[:, None] + 1 + np.arange(8)[None, :]) % n)
    assert np.array_equal(engine.chord_fingers(), OracleNet("chord", net.ids, net.xy).chord_fingers())


# ------------------------------------------------------------ extendedFingerTable (Chord.cc:416-419, 627-641)

@pytest.mark.parametrize("nfc,rt", [(3, 0), (1, 0), (8, 0), (3, 1)])
def test_extended_finger_table_matches_oracle(engine: KbrEngine, nfc, rt):
    """With no FindNodeCall able to time out (150 x 150 coordinate field: RTT <= ~0.43 s against
    rpcUdpTimeout 1.5 s), the engine routes with extendedFingerTable = true and equals the oracle,
    which restates the finger candidate lists (tests/test_oracle_extended.py)."""
    net = W.population(1 << 14, 41)
    p = Params.chord().replace(extendedFingerTable=1, numFingerCandidates=nfc, routingType=rt)
    engine.set_params(p)
    engine.chord_load(net.ids, net.xy)
    o = OracleNet("chord", net.ids, net.xy, chord_params(extendedFingerTable=1, numFingerCandidates=nfc, routingType=rt))
    k1, s1 = W.lookups(net.ids, 3000, 42, node_ids=True)
    k2, s2 = W.lookups(net.ids, 3000, 43, node_ids=False)
    keys, src = np.concatenate([k1, k2]), np.concatenate([s1, s2])
    _eq(engine.lookup(keys, src, record_hops=True), o.route(keys, src, record_hops=True), f"extended nfc={nfc} rt={rt}",
        hop_cols=50)
    if rt == 0:
        g, r = engine.lookupCall(keys, src), o.lookup_call(keys, src)
        for f in ("num_siblings", "hops", "status", "is_valid", "latency_ns"):
            assert np.array_equal(np.asarray(g[f]).astype(np.int64), np.asarray(r[f]).astype(np.int64)), f


def test_extended_finger_table_refusals(engine: KbrEngine):
    """Refused where the extended table would route differently or answer lists the engine does not
    build: a FindNodeCall that could time out (the next start candidate would be tried), findNode
    answers of more than one node, explicit tables."""
    from oversim_amd import KbrError
    net = W.population(2000, 44)
    k, s = W.lookups(net.ids, 500, 45, node_ids=False)
    engine.set_params(Params.chord().replace(extendedFingerTable=1, rpcUdpTimeout=0.25))
    engine.chord_load(net.ids, net.xy)
    with pytest.raises(KbrError, match="time out"):
        engine.lookup(k, s)
    # recursive routes carry no RPC timeout: accepted, equal to the oracle
    engine.set_params(Params.chord().replace(extendedFingerTable=1, rpcUdpTimeout=0.25, routingType=1))
    o = OracleNet("chord", net.ids, net.xy, chord_params(extendedFingerTable=1, rpcUdpTimeout=0.25, routingType=1))
    _eq(engine.lookup(k, s, record_hops=True), o.route(k, s, record_hops=True), "extended recursive", hop_cols=50)
    engine.set_params(Params.chord().replace(extendedFingerTable=1))
    nodes, cnt, sib = engine.findNode(s[:10], k[:10], 1, 1)          # one node: the non-extended finger
    o1 = OracleNet("chord", net.ids, net.xy, chord_params(extendedFingerTable=1))
    for i in range(10):
        assert list(nodes[i, :cnt[i]]) == o1.find_node(int(s[i]), k[i], 1, 1)[0]
    with pytest.raises(KbrError, match="extendedFingerTable"):
        engine.findNode(s[:10], k[:10], 3, 1)
    fingers = OracleNet("chord", net.ids, net.xy).chord_fingers()
    n = len(net.ids)
    engine.set_params(Params.chord())
    engine.chord_load_tables(net.ids, net.xy, ((np.arange(n) - 1) % n).astype(np.uint32),
                             ((np.arange(n)[:, None] + 1 + np.arange(8)[None, :]) % n).astype(np.uint32),
                             np.full(n, 8, np.uint8), fingers, np.full(n, 160, np.uint8))
    engine.set_params(Params.chord().replace(extendedFingerTable=1))
    with pytest.raises(KbrError, match="explicit tables"):
        engine.lookup(k, s)


def test_key_order_matches_caller_order(engine: KbrEngine, monkeypatch):
    """K1 key order (ksort.hip): a batch routed in the order of its keys' top bits, every result and
    hop sequence written at its caller index, equals the batch routed in caller order and the golden
    vectors.  The key order is opt-in: OVS_K1_SORT=1 and OVS_K1_SORT_MIN (default 2^20 lookups), read
    per call."""
    g = np.load(GOLD / "chord_n1000_round.npz")
    engine.set_params(Params.chord())
    engine.chord_load(g["ids"], g["xy"])
    monkeypatch.setenv("OVS_K1_SORT", "1")
    monkeypatch.setenv("OVS_K1_SORT_MIN", "1")
    r = engine.lookup(g["keys"], g["src"], record_hops=True)
    H = g["hop_seq"].shape[1]
    _eq(r, {f: g[f] for f in FIELDS} | {"hop_seq": g["hop_seq"]}, "key order, golden", hop_cols=H)
    net = W.population(1 << 20, 0x50F)
    engine.chord_load(net.ids, net.xy)
    keys, src = W.lookups(net.ids, 1 << 21, 0x510, node_ids=False)
    keys[:4096] = net.ids[src[:4096]]          # node-ID keys and equal keys land in the same bins
    keys[4096:8192] = keys[0]
    monkeypatch.setenv("OVS_K1_SORT_MIN", "1")
    a = engine.lookup(keys, src)
    monkeypatch.setenv("OVS_K1_SORT_MIN", str(1 << 40))
    b = engine.lookup(keys, src)
    _eq(a, b, "key order vs caller order")
    o = OracleNet("chord", net.ids, net.xy).route(keys[:50000], src[:50000], record_hops=False)
    _eq({f: a[f][:50000] for f in FIELDS}, o, "key order vs oracle")
