"""Generate the committed golden vectors under tests/golden/.

Provenance: the reference (trucndt/oversim) needs OMNeT++ 4.x + INET and cannot
be built in this image, and ships no routing fixtures.  These vectors are
therefore produced by the CPU restatement in oracle/ (ovs_oracle.c) and, for
every case, re-derived independently by tests/refmodel.py before being written (Chord: a direct
alpha = 1 loop; Kademlia: findNode on its own KadTables and the lookup as a message-level
discrete-event simulation, KadLookupSim); a disagreement aborts generation.  They freeze the restated
reference semantics so that regressions of either the oracle or the engine
are caught.  Inputs (IDs, coordinates, keys, sources) come from the seeded
generator in oversim_amd/workload.py; coordinates for N <= 15000 are records of
the reference's simulations/nodes_2d_15000.xml.

Each .npz records the SimTime rounding rule it was generated with.
Run: python tests/golden/make_golden.py [--kad] [--rec] [--auth] [--kadrec] [--koorde] [--check: with --koorde verify the
committed Koorde vectors, alone the committed Kademlia vectors, instead of rewriting them]
"""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent.parent))
sys.path.insert(0, str(HERE.parent))

from oversim_amd import workload as W  # noqa: E402
from oracle_lib import OracleNet, chord_params, kad_params, koorde_params  # noqa: E402
import refmodel  # noqa: E402


def chord_case(name: str, n: int, seed: int, m_ids: int, m_rand: int, rnd: int, auth: int = 0):
    """auth: measureAuthBlock = true -- every FindNodeResponse 100 B longer (AUTHBLOCK_L,
    CommonMessages.msg:45-47, 57, 73)."""
    net = W.population(n, seed)
    k1, s1 = W.lookups(net.ids, m_ids, seed + 1, node_ids=True)
    k2, s2 = W.lookups(net.ids, m_rand, seed + 2, node_ids=False)
    keys = np.concatenate([k1, k2])
    src = np.concatenate([s1, s2])
    o = OracleNet("chord", net.ids, net.xy, chord_params(simtimeRound=rnd, measureAuthBlock=auth))
    r = o.route(keys, src, record_hops=True)
    ring = refmodel.ChordRing(net.ids, net.xy, rnd=bool(rnd))
    for i in range(len(keys)):
        m = ring.lookup(keys[i], int(src[i]), resp=87 + 100 * auth)
        for f in ("responsible", "hops", "status", "one_way_hops", "latency_ns"):
            assert int(r[f][i]) == int(m[f]), (name, i, f, r[f][i], m[f])
        assert [int(x) for x in r["hop_seq"][i] if x != 0xFFFFFFFF] == m["hop_seq"], (name, i)
    H = int(r["hops"].max()) + 1
    np.savez_compressed(HERE / f"{name}.npz", ids=net.ids, xy=net.xy, keys=keys, src=src,
                        responsible=r["responsible"], hops=r["hops"], status=r["status"],
                        one_way_hops=r["one_way_hops"], latency_ns=r["latency_ns"],
                        hop_seq=r["hop_seq"][:, :H], simtime_round=np.int32(rnd), seed=np.int64(seed),
                        measure_auth_block=np.int32(auth))
    print(name, "lookups", len(keys), "mean hops", r["hops"].mean(), "status", np.bincount(r["status"]))


def chord_rec_case(name: str, n: int, seed: int, m_ids: int, m_rand: int, rnd: int, hcm: int = 50):
    """Semi-recursive routing (routingType = semi-recursive, ChordLarge), checked against
    refmodel.ChordRing.lookup_recursive before writing."""
    net = W.population(n, seed)
    k1, s1 = W.lookups(net.ids, m_ids, seed + 1, node_ids=True)
    k2, s2 = W.lookups(net.ids, m_rand, seed + 2, node_ids=False)
    keys = np.concatenate([k1, k2])
    src = np.concatenate([s1, s2])
    o = OracleNet("chord", net.ids, net.xy, chord_params(simtimeRound=rnd, routingType=1, hopCountMax=hcm))
    r = o.route(keys, src, record_hops=True)
    ring = refmodel.ChordRing(net.ids, net.xy, rnd=bool(rnd))
    for i in range(len(keys)):
        m = ring.lookup_recursive(keys[i], int(src[i]), hop_max=hcm)
        for f in ("responsible", "hops", "status", "one_way_hops", "latency_ns"):
            assert int(r[f][i]) == int(m[f]), (name, i, f, r[f][i], m[f])
    H = int(r["hops"].max()) + 1
    np.savez_compressed(HERE / f"{name}.npz", ids=net.ids, xy=net.xy, keys=keys, src=src,
                        responsible=r["responsible"], hops=r["hops"], status=r["status"],
                        one_way_hops=r["one_way_hops"], latency_ns=r["latency_ns"],
                        hop_seq=r["hop_seq"][:, :H], simtime_round=np.int32(rnd), seed=np.int64(seed),
                        routing_type=np.int32(1), hop_count_max=np.int32(hcm))
    print(name, "lookups", len(keys), "mean hops", r["hops"].mean(), "status", np.bincount(r["status"]))


def kad_case(name: str, n: int, seed: int, m: int, alpha: int, rnd: int = 1, **kw):
    """kw: further Kademlia parameters ([Config KademliaLarge]: k = lookupRedundantNodes = 16)."""
    net = W.population(n, seed)
    k1, s1 = W.lookups(net.ids, m, seed + 1, node_ids=True)
    p = kad_params(lookupParallelRpcs=alpha, simtimeRound=rnd, **kw)
    R = p.lookupRedundantNodes
    o = OracleNet("kademlia", net.ids, net.xy, p)
    sib, cnt, nodes = o.kad_tables()
    # findNode restated twice: oracle vs refmodel on the oracle's own snapshot
    tab = refmodel.KadTables(net.ids, sib, cnt, nodes, k=p.k, s=p.s)
    rng = np.random.default_rng(seed + 3)
    fn_node = rng.integers(0, n, 512).astype(np.uint32)
    fn_key = np.concatenate([W.random_keys(256, rng), net.ids[rng.integers(0, n, 256)]])
    fn_out = np.full((512, max(R, 8)), 0xFFFFFFFF, dtype=np.uint32)
    fn_sib = np.zeros(512, dtype=np.uint8)
    for i in range(512):
        res, flag = o.find_node(int(fn_node[i]), fn_key[i], R, 1)
        ref = tab.find_node(int(fn_node[i]), refmodel.to_int(fn_key[i]), R, 1)
        assert [int(x) for x in res] == ref, (name, i, res, ref)
        assert flag == tab.is_sibling_for(int(fn_node[i]), refmodel.to_int(fn_key[i]), 1)
        fn_out[i, :len(res)] = res
        fn_sib[i] = flag
    r = o.route(k1, s1, record_hops=True, count_rpcs=True)
    # the lookups restated twice: oracle event list vs refmodel's message-level simulation
    sim = refmodel.KadLookupSim(tab, net.xy, redundant=R, alpha=alpha, rnd=bool(rnd), k=p.k,
                                resp_base=61 + 100 * p.measureAuthBlock)
    for i in range(len(k1)):
        mm = sim.run(k1[i], int(s1[i]))
        for f in ("responsible", "hops", "status", "one_way_hops", "latency_ns", "rpcs"):
            assert int(r[f][i]) == int(mm[f]), (name, i, f, r[f][i], mm[f])
        assert [int(x) for x in r["hop_seq"][i] if x != 0xFFFFFFFF] == mm["hop_seq"], (name, i)
    H = int(r["hops"].max()) + 1
    if "--check" in sys.argv:
        g = np.load(HERE / f"{name}.npz")
        for f in ("responsible", "hops", "status", "one_way_hops", "latency_ns", "rpcs", "fn_out", "fn_sib"):
            assert np.array_equal(g[f], {**r, "fn_out": fn_out, "fn_sib": fn_sib}[f]), (name, f)
        assert np.array_equal(g["hop_seq"], r["hop_seq"][:, :H]), name
        print(name, "committed vectors reproduced")
        return
    np.savez_compressed(HERE / f"{name}.npz", ids=net.ids, xy=net.xy, keys=k1, src=s1, alpha=np.int32(alpha),
                        responsible=r["responsible"], hops=r["hops"], status=r["status"],
                        one_way_hops=r["one_way_hops"], latency_ns=r["latency_ns"], rpcs=r["rpcs"],
                        hop_seq=r["hop_seq"][:, :H], simtime_round=np.int32(rnd), seed=np.int64(seed),
                        kad_seed=np.uint64(p.kadSeed), fn_node=fn_node, fn_key=fn_key, fn_out=fn_out,
                        fn_sib=fn_sib, k=np.int32(p.k), s=np.int32(p.s), redundant=np.int32(R),
                        measure_auth_block=np.int32(p.measureAuthBlock))
    print(name, "lookups", len(k1), "mean hops", r["hops"].mean(), "rpcs", r["rpcs"].mean(),
          "status", np.bincount(r["status"]))


def koorde_case(name: str, n: int, seed: int, m_ids: int, m_rand: int, **kw):
    """Koorde one-way lookups (iterative, Koorde defaults unless overridden), checked against
    refmodel.KoordeRing (a second reading of Koorde.cc) before writing."""
    net = W.population(n, seed)
    k1, s1 = W.lookups(net.ids, m_ids, seed + 1, node_ids=True)
    k2, s2 = W.lookups(net.ids, m_rand, seed + 2, node_ids=False)
    keys, src = np.concatenate([k1, k2]), np.concatenate([s1, s2])
    p = koorde_params(**kw)
    o = OracleNet("koorde", net.ids, net.xy, p)
    r = o.route(keys, src, record_hops=True, count_rpcs=True)
    ring = refmodel.KoordeRing(net.ids, net.xy, p.successorListSize, p.deBruijnListSize, p.shiftingBits,
                               bool(p.useOtherLookup), bool(p.useSucList))
    for i in range(len(keys)):
        m = ring.lookup(keys[i], int(src[i]))
        for f in ("responsible", "hops", "status", "one_way_hops", "latency_ns"):
            assert int(r[f][i]) == int(m[f]), (name, i, f, r[f][i], m[f])
        assert [int(x) for x in r["hop_seq"][i] if x != 0xFFFFFFFF] == m["hop_seq"], (name, i)
    db, dstart, dnum = o.koorde_state()
    H = int(r["hops"].max()) + 1
    out = dict(responsible=r["responsible"], hops=r["hops"], status=r["status"], one_way_hops=r["one_way_hops"],
               latency_ns=r["latency_ns"], rpcs=r["rpcs"], hop_seq=r["hop_seq"][:, :H], db=db, db_start=dstart,
               db_num=dnum)
    if "--check" in sys.argv:
        g = np.load(HERE / f"{name}.npz")
        for f, v in out.items():
            assert np.array_equal(g[f], v), (name, f)
        print(name, "committed vectors reproduced")
        return
    np.savez_compressed(HERE / f"{name}.npz", ids=net.ids, xy=net.xy, keys=keys, src=src, seed=np.int64(seed),
                        successorListSize=np.int32(p.successorListSize), deBruijnListSize=np.int32(p.deBruijnListSize),
                        shiftingBits=np.int32(p.shiftingBits), useOtherLookup=np.int32(p.useOtherLookup),
                        useSucList=np.int32(p.useSucList), **out)
    print(name, "lookups", len(keys), "mean hops", r["hops"].mean(), "status", np.bincount(r["status"]))


def kad_rec_case(name: str, n: int, seed: int, m: int, rnd: int = 1, hcm: int = 50, **kw):
    """R/Kademlia: recursive one-way routes (semi- and full-recursive route a KBRTestMessage the same
    way) and recursive LookupCalls (numSiblings 1, s, 0; semi- and full-recursive responses) over
    the snapshot tables, checked against refmodel.KadRecursiveSim before writing."""
    net = W.population(n, seed)
    k1, s1 = W.lookups(net.ids, m // 2, seed + 1, node_ids=True)
    k2, s2 = W.lookups(net.ids, m // 2, seed + 2, node_ids=False)
    keys, src = np.concatenate([k1, k2]), np.concatenate([s1, s2])
    out = {}
    for rt in (1, 2):
        p = kad_params(routingType=rt, simtimeRound=rnd, hopCountMax=hcm, **kw)
        o = OracleNet("kademlia", net.ids, net.xy, p)
        sib, cnt, nodes = o.kad_tables()
        sim = refmodel.KadRecursiveSim(refmodel.KadTables(net.ids, sib, cnt, nodes, k=p.k, s=p.s), net.xy, k=p.k,
                                       s=p.s, rec_redundant=p.recNumRedundantNodes, redundant=p.lookupRedundantNodes,
                                       hop_max=hcm, rnd=bool(rnd))
        if rt == 1:
            r = o.route(keys, src, record_hops=True)
            for i in range(len(keys)):
                mm = sim.route(keys[i], int(src[i]))
                for f in ("responsible", "hops", "status", "latency_ns"):
                    assert int(r[f][i]) == int(mm[f]), (name, i, f, r[f][i], mm[f])
                assert [int(x) for x in r["hop_seq"][i] if x != 0xFFFFFFFF] == mm["hop_seq"], (name, i)
            H = int(r["hops"].max()) + 1
            out.update(responsible=r["responsible"], hops=r["hops"], status=r["status"],
                       one_way_hops=r["one_way_hops"], latency_ns=r["latency_ns"], hop_seq=r["hop_seq"][:, :H])
        for ns in (1, p.s, 0):
            lc = o.lookup_call(keys, src, ns)
            for i in range(len(keys)):
                mm = sim.lookup_call(keys[i], int(src[i]), ns, full=(rt == 2))
                for f in ("num_siblings", "hops", "status", "is_valid", "latency_ns"):
                    assert int(lc[f][i]) == int(mm[f]), (name, rt, ns, i, f, lc[f][i], mm[f])
                assert [int(x) for x in lc["siblings"][i] if x != 0xFFFFFFFF] == mm["siblings"][:max(ns, 1)], (name, i)
            for f in ("num_siblings", "status", "is_valid", "latency_ns", "siblings"):
                out[f"lc{rt}_ns{ns}_{f}"] = np.asarray(lc[f])
    if "--check" in sys.argv:
        g = np.load(HERE / f"{name}.npz")
        for f, v in out.items():
            assert np.array_equal(g[f], v), (name, f)
        print(name, "committed vectors reproduced")
        return
    np.savez_compressed(HERE / f"{name}.npz", ids=net.ids, xy=net.xy, keys=keys, src=src, seed=np.int64(seed),
                        simtime_round=np.int32(rnd), hop_count_max=np.int32(hcm), **out)
    print(name, "lookups", len(keys), "mean hops", out["hops"].mean(), "status", np.bincount(out["status"]),
          "lookup-call valid", out["lc1_ns8_is_valid"].mean(), out["lc2_ns8_is_valid"].mean())


def src_route_case(name: str, n_chord: int, n_kad: int, seed: int, m: int, rnd: int = 1):
    """routingType = "source-routing-recursive" (BaseOverlay.cc:129-130; verify.ini [Config ChordSource]).
    One-way routes on Chord and Kademlia: the route message records its senders and skips them in the
    loop detection, its length stays the one set at creation (BaseOverlay.cc:888-897, 1398, 1502-1516),
    so on converged rings and snapshot tables the routes equal semi-recursive ones -- the oracle is
    checked against its own semi-recursive routes and against refmodel.  Kademlia LookupCalls: the
    response travels back along the call's recorded route, reversed (BaseRpc.cc:575-588), with the
    R/Kademlia hook at every node on the way -- oracle vs refmodel.KadRecursiveSim(source_routing)."""
    out = {}
    # Chord
    net = W.population(n_chord, seed)
    k1, s1 = W.lookups(net.ids, m // 2, seed + 1, node_ids=True)
    k2, s2 = W.lookups(net.ids, m // 2, seed + 2, node_ids=False)
    keys, src = np.concatenate([k1, k2]), np.concatenate([s1, s2])
    r4 = OracleNet("chord", net.ids, net.xy, chord_params(simtimeRound=rnd, routingType=4)).route(keys, src, record_hops=True)
    r1 = OracleNet("chord", net.ids, net.xy, chord_params(simtimeRound=rnd, routingType=1)).route(keys, src, record_hops=True)
    ring = refmodel.ChordRing(net.ids, net.xy, rnd=bool(rnd))
    for f in ("responsible", "hops", "status", "one_way_hops", "latency_ns", "hop_seq"):
        assert np.array_equal(r4[f], r1[f]), (name, "chord: source routing differs from semi-recursive", f)
    for i in range(len(keys)):
        mm = ring.lookup_recursive(keys[i], int(src[i]))
        for f in ("responsible", "hops", "status", "one_way_hops", "latency_ns"):
            assert int(r4[f][i]) == int(mm[f]), (name, i, f, r4[f][i], mm[f])
    H = int(r4["hops"].max()) + 1
    out.update(chord_ids=net.ids, chord_xy=net.xy, chord_keys=keys, chord_src=src,
               **{f"chord_{f}": r4[f] for f in ("responsible", "hops", "status", "one_way_hops", "latency_ns")},
               chord_hop_seq=r4["hop_seq"][:, :H])
    # Kademlia
    net = W.population(n_kad, seed + 10)
    k1, s1 = W.lookups(net.ids, m // 2, seed + 11, node_ids=True)
    k2, s2 = W.lookups(net.ids, m // 2, seed + 12, node_ids=False)
    keys, src = np.concatenate([k1, k2]), np.concatenate([s1, s2])
    p = kad_params(routingType=4, simtimeRound=rnd)
    o = OracleNet("kademlia", net.ids, net.xy, p)
    sib, cnt, nodes = o.kad_tables()
    sim = refmodel.KadRecursiveSim(refmodel.KadTables(net.ids, sib, cnt, nodes, k=p.k, s=p.s), net.xy, k=p.k, s=p.s,
                                   rec_redundant=p.recNumRedundantNodes, redundant=p.lookupRedundantNodes, rnd=bool(rnd))
    r = o.route(keys, src, record_hops=True)
    r1 = OracleNet("kademlia", net.ids, net.xy, kad_params(routingType=1, simtimeRound=rnd)).route(keys, src,
                                                                                                   record_hops=True)
    for f in ("responsible", "hops", "status", "one_way_hops", "latency_ns", "hop_seq"):
        assert np.array_equal(r[f], r1[f]), (name, "kademlia: source routing differs from semi-recursive", f)
    for i in range(len(keys)):
        mm = sim.route(keys[i], int(src[i]), source_routing=True)
        for f in ("responsible", "hops", "status", "latency_ns"):
            assert int(r[f][i]) == int(mm[f]), (name, i, f, r[f][i], mm[f])
    H = int(r["hops"].max()) + 1
    out.update(kad_ids=net.ids, kad_xy=net.xy, kad_keys=keys, kad_src=src,
               **{f"kad_{f}": r[f] for f in ("responsible", "hops", "status", "one_way_hops", "latency_ns")},
               kad_hop_seq=r["hop_seq"][:, :H])
    for ns in (1, p.s, 0):
        lc = o.lookup_call(keys, src, ns)
        for i in range(len(keys)):
            mm = sim.lookup_call(keys[i], int(src[i]), ns, source_routing=True)
            for f in ("num_siblings", "hops", "status", "is_valid", "latency_ns"):
                assert int(lc[f][i]) == int(mm[f]), (name, ns, i, f, lc[f][i], mm[f])
            assert [int(x) for x in lc["siblings"][i] if x != 0xFFFFFFFF] == mm["siblings"][:max(ns, 1)], (name, i)
        for f in ("num_siblings", "status", "is_valid", "latency_ns", "siblings"):
            out[f"kad_lc_ns{ns}_{f}"] = np.asarray(lc[f])
    if "--check" in sys.argv:
        g = np.load(HERE / f"{name}.npz")
        for f, v in out.items():
            assert np.array_equal(g[f], v), (name, f)
        print(name, "committed vectors reproduced")
        return
    np.savez_compressed(HERE / f"{name}.npz", seed=np.int64(seed), simtime_round=np.int32(rnd),
                        routing_type=np.int32(4), **out)
    print(name, "chord mean hops", out["chord_hops"].mean(), "kad mean hops", out["kad_hops"].mean(),
          "lookup-call valid", out["kad_lc_ns8_is_valid"].mean())


if __name__ == "__main__":
    if "--srcroute" in sys.argv:   # (with --check: verify instead of writing)
        src_route_case("srcroute_n2000", 1000, 2000, 0x5C0, 2048)
        sys.exit(0)
    if "--kadrec" in sys.argv:   # (with --check: verify instead of writing)
        kad_rec_case("kad_n2000_rec", 2000, 0x4b52, 2048)
        kad_rec_case("kad_n1000_rec_hcm3", 1000, 0x4b53, 1024, rnd=0, hcm=3)
        sys.exit(0)
    if "--koorde" in sys.argv:   # (with --check: verify instead of writing)
        koorde_case("koorde_n2000", 2000, 0x4b4f, 1024, 1024)
        koorde_case("koorde_n2000_sb2_nosuc", 2000, 0x4b50, 512, 512, shiftingBits=2, useSucList=0)
        sys.exit(0)
    if "--auth" in sys.argv:   # measureAuthBlock = true (default.ini:399 flipped), Chord and Kademlia alpha 3
        chord_case("chord_n1000_auth", 1000, 0x4215, 2048, 2048, 1, auth=1)
        kad_case("kad_n2000_a3_auth", 2000, 0x4b44, 2048, 3, measureAuthBlock=1)
        sys.exit(0)
    if "--rec" in sys.argv:
        chord_rec_case("chord_n1000_semirec", 1000, 0x4213, 2048, 2048, 1)
        chord_rec_case("chord_n1000_semirec_hcm4", 1000, 0x4214, 512, 512, 0, hcm=4)
        sys.exit(0)
    if "--large" in sys.argv:   # [Config KademliaLarge] (omnetpp.ini:113-126), 1000 nodes as configured
        kad_case("kad_n1000_large", 1000, 0x4b4c, 2048, 1, k=16, lookupRedundantNodes=16, s=8)
        kad_case("kad_n1000_large_a3", 1000, 0x4b4d, 1024, 3, k=16, lookupRedundantNodes=16, s=8)
        sys.exit(0)
    if "--check" in sys.argv and "--koorde" not in sys.argv:
        kad_case("kad_n2000_a1", 2000, 0x4b41, 2048, 1)
        kad_case("kad_n2000_a3", 2000, 0x4b41, 2048, 3)
        sys.exit(0)
    chord_case("chord_n1000_round", 1000, 0x4213, 4096, 4096, 1)
    chord_case("chord_n1000_trunc", 1000, 0x4213, 2048, 2048, 0)
    chord_case("chord_n9", 9, 5, 256, 256, 1)
    chord_case("chord_n2", 2, 6, 64, 64, 1)
    if "--kad" in sys.argv:
        kad_case("kad_n2000_a1", 2000, 0x4b41, 2048, 1)
        kad_case("kad_n2000_a3", 2000, 0x4b41, 2048, 3)
