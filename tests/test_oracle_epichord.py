"""EpiChord::findNode: the oracle restatement (oracle/ovs_oracle_epichord.c) against the independent
second reading in tests/refmodel.py, on generated routing snapshots (tests/epichord_snap.py).
Parity unpinned against reference outputs (no EpiChord fixtures in the reference, which cannot be
built here)."""
from __future__ import annotations

import numpy as np
import pytest

import refmodel as RM
from epichord_snap import NONE, make_queries, make_snapshot
from oracle_lib import epichord_find_node


def _ref(snap, keys_int, v, key, src, now, R):
    o0, o1 = int(snap["cache_off"][v]), int(snap["cache_off"][v + 1])
    cache = {int(x): (int(lu), int(t)) for x, lu, t in zip(snap["cache_node"][o0:o1], snap["cache_last"][o0:o1],
                                                           snap["cache_ttl"][o0:o1])}
    succ = [int(x) for x in snap["succ"][v, :snap["nsucc"][v]]]
    pred = [int(x) for x in snap["pred"][v, :snap["npred"][v]]]
    return RM.epichord_find_node(keys_int, v, succ, pred, int(snap["full"][v]), snap["L"], cache, RM.to_int(key),
                                 None if src == NONE else int(src), int(now), snap["cache_ttl_param"], R)


@pytest.mark.parametrize("n,L,R,seed", [(2, 4, 3, 1), (3, 4, 3, 2), (5, 4, 3, 3), (40, 4, 3, 4), (300, 4, 3, 5),
                                        (300, 8, 5, 6), (1000, 2, 1, 7), (1000, 4, 16, 8)])
def test_oracle_matches_refmodel(n, L, R, seed):
    snap = make_snapshot(n, seed, list_size=L)
    keys_int = [RM.to_int(k) for k in snap["ids"]]
    node, keys, src, now = make_queries(snap, 600, seed + 100)
    seen = {0: 0, -1: 0, -2: 0, "sib": 0}
    for i in range(len(node)):
        r, nodes, lasts = epichord_find_node(snap, int(node[i]), keys[i], int(src[i]), int(now[i]), R)
        st, ref = _ref(snap, keys_int, int(node[i]), keys[i], int(src[i]), int(now[i]), R)
        if st < 0:
            assert r == st, (i, r, st)
        else:
            assert r == len(ref), (i, r, ref)
        seen[min(r, 0) if r <= 0 else 0] += 1
        got = list(zip(nodes.tolist(), lasts.tolist()))
        assert got == [(int(x), int(t)) for x, t in ref][:max(r, 0)], (i, got, ref)
        if r > 0 and nodes[0] == node[i]:
            seen["sib"] += 1
    assert seen[0] > 0 and seen["sib"] > 0
