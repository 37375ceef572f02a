"""CPU: the oracle's Chord exact-key LookupCalls (numSiblings = 0) against a second reading of the
rules.  The oracle runs the literal IterativeLookup (IterativeLookup.cc:157-184, 803-921) over
Chord::findNode, whose responsible node answers nothing when numSiblings = 0 (Chord.cc:573-580,
downsizeTo(0)).  Read from the one-way route instead: findNode's choice elsewhere does not depend on
numSiblings, so the lookup walks the route's chain R1..Rk (Rk responsible) and succeeds at the
response that names the key's node -- response k-1, which needs k >= 2 -- and otherwise fails after
response k (0 hops when the source is responsible itself)."""
from __future__ import annotations

import numpy as np

from oracle_lib import OracleNet
from oversim_amd import workload as W


def test_chord_exact_key_lookups_follow_the_route_chain():
    net = W.population(3000, 71)
    o = OracleNet("chord", net.ids, net.xy)
    k1, s1 = W.lookups(net.ids, 2000, 72, node_ids=True)
    k2, s2 = W.lookups(net.ids, 1000, 73, node_ids=False)
    keys, src = np.concatenate([k1, k2]), np.concatenate([s1, s2])
    e = o.lookup_call(keys, src, 0)
    r = o.route(keys, src)
    assert np.all(r["status"] == 0)                        # a converged ring: every route succeeds
    k = r["hops"].astype(np.int64)
    found = np.zeros(len(keys), dtype=bool)
    found[:2000] = k[:2000] >= 2
    assert np.array_equal(e["is_valid"] == 1, found)
    assert np.array_equal(e["hops"][found].astype(np.int64), k[found] - 1)
    assert np.array_equal(e["hops"][~found].astype(np.int64), k[~found])
    assert np.array_equal(e["siblings"][found, 0], r["responsible"][found])
    assert np.all(e["num_siblings"][found] == 1) and np.all(e["num_siblings"][~found] == 0)
    assert found.sum() > 1500
