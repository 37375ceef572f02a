"""Koorde (src/overlay/koorde/Koorde.cc) restated twice: the oracle (ovs_oracle.c, literal
interval loops, the extension threaded through IterativeLookup) and refmodel.KoordeRing (Python
integers, list walks by clockwise distance).  CPU only: the two readings agree on the de Bruijn
state and on whole lookups over parameter variants, and the oracle reproduces the committed
Koorde golden vectors (tests/golden/koorde_*.npz, generated with both readings in agreement)."""
from __future__ import annotations

from pathlib import Path

import numpy as np
import pytest

import refmodel
from oracle_lib import OracleNet, koorde_params
from oversim_amd import Params, workload as W

GOLD = Path(__file__).resolve().parent / "golden"
FIELDS = ("responsible", "hops", "status", "one_way_hops", "latency_ns")


@pytest.mark.parametrize("n,sls,dbls,sb,uo,us,seed", [
    (40, 16, 16, 4, 1, 1, 1), (1500, 16, 16, 4, 1, 1, 2), (1500, 8, 16, 4, 1, 1, 3), (1500, 16, 8, 2, 1, 1, 4),
    (1500, 16, 16, 4, 0, 1, 5), (1500, 16, 16, 4, 1, 0, 6), (1500, 4, 4, 3, 1, 1, 7), (12, 16, 16, 4, 1, 1, 8),
    (2500, 16, 16, 8, 1, 1, 9), (1500, 16, 16, 1, 1, 1, 10),
])
def test_oracle_agrees_with_refmodel(n, sls, dbls, sb, uo, us, seed):
    net = W.population(n, seed)
    p = koorde_params(successorListSize=sls, deBruijnListSize=dbls, shiftingBits=sb, useOtherLookup=uo, useSucList=us)
    o = OracleNet("koorde", net.ids, net.xy, p)
    R = refmodel.KoordeRing(net.ids, net.xy, sls, dbls, sb, bool(uo), bool(us))
    db, st, num = o.koorde_state()
    for v in range(n):
        dbn, dbl = R.db[v]
        assert (db[v], st[v], num[v]) == (dbn, dbl[0], len(dbl)), v
    k1, s1 = W.lookups(net.ids, 300, seed + 10, node_ids=True)
    k2, s2 = W.lookups(net.ids, 300, seed + 11, node_ids=False)
    keys, src = np.concatenate([k1, k2]), np.concatenate([s1, s2])
    r = o.route(keys, src, record_hops=True)
    for i in range(len(keys)):
        m = R.lookup(keys[i], int(src[i]))
        for f in FIELDS:
            assert int(r[f][i]) == int(m[f]), (i, f, r[f][i], m[f])
        assert [int(x) for x in r["hop_seq"][i] if x != 0xFFFFFFFF] == m["hop_seq"], i


@pytest.mark.parametrize("name", ["koorde_n2000", "koorde_n2000_sb2_nosuc"])
def test_oracle_reproduces_koorde_golden(name):
    g = np.load(GOLD / f"{name}.npz")
    p = koorde_params(successorListSize=int(g["successorListSize"]), deBruijnListSize=int(g["deBruijnListSize"]),
                      shiftingBits=int(g["shiftingBits"]), useOtherLookup=int(g["useOtherLookup"]),
                      useSucList=int(g["useSucList"]))
    o = OracleNet("koorde", g["ids"], g["xy"], p)
    r = o.route(g["keys"], g["src"], record_hops=True, count_rpcs=True)
    for f in FIELDS + ("rpcs",):
        assert np.array_equal(r[f].astype(np.int64), g[f].astype(np.int64)), f
    assert np.array_equal(r["hop_seq"][:, :g["hop_seq"].shape[1]], g["hop_seq"])
    db, st, num = o.koorde_state()
    assert np.array_equal(db, g["db"]) and np.array_equal(st, g["db_start"]) and np.array_equal(num, g["db_num"])


def test_find_node_throws_like_the_reference():
    """findDeBruijnHop's bounding error (step > keyLength) and a getBit below bit 0 are
    cRuntimeErrors in the reference (Koorde.cc:490-493, OverlayKey::getBitRange)."""
    net = W.population(500, 3)
    o = OracleNet("koorde", net.ids, net.xy)
    rng = np.random.default_rng(4)
    thrown = 0
    for _ in range(400):
        v = int(rng.integers(0, 500))
        key = W.random_keys(1, rng)[0]
        h, rk, step = o.koorde_find_node(v, key)
        if h is None:
            continue
        # replay with an extension whose step is past the key length: any de Bruijn step throws
        h2, _, _ = o.koorde_find_node(v, key, rk if rk is not None else np.zeros(5, np.uint32), 161)
        thrown += h2 is None
    assert thrown > 0


def test_koorde_params_mirror_the_engine_defaults():
    """ovs_params_default(OVS_OVERLAY_KOORDE) and orc_params_koorde_default: default.ini:268-291."""
    e, o = Params.koorde(), koorde_params()
    for f in ("successorListSize", "shiftingBits", "deBruijnListSize", "useOtherLookup", "useSucList",
              "lookupRedundantNodes", "lookupParallelRpcs", "lookupMerge", "hopCountMax"):
        assert getattr(e, f) == getattr(o, f), f
    assert (e.successorListSize, e.shiftingBits, e.deBruijnListSize) == (16, 4, 16)
