"""Multi-round Chord convergence in the oracle (CPU): a ring whose older nodes do not know the
nodes that joined last (their successor lists and predecessors skip them; the joined nodes know
their successors but no predecessor) reaches the stable ring's tables -- predecessors, successor
lists and fingers -- by alternating synchronous stabilize rounds (Chord.cc:793-842, 1055-1225) and
fixfingers rounds (845-875, 1228-1270)."""
from __future__ import annotations

import numpy as np

from oversim_amd import workload as W
from oracle_lib import OracleNet, chord_params

NONE = 0xFFFFFFFF


def joined_ring(n: int, seed: int, frac: float = 0.1, sls: int = 8):
    """Tables as the old members hold them after a batch of joins: the joined nodes are invisible
    to the old members' successor lists, predecessors and fingers; a joined node knows its true
    successor list (its join response) and no predecessor."""
    net = W.population(n, seed)
    rng = np.random.default_rng(seed)
    joined = np.zeros(n, dtype=bool)
    joined[rng.choice(n, int(n * frac), replace=False)] = True
    old = np.nonzero(~joined)[0]
    pos = np.searchsorted(old, np.arange(n))            # index of the first old node >= v
    succ = np.full((n, sls), NONE, dtype=np.uint32)
    pred = np.full(n, NONE, dtype=np.uint32)
    for v in range(n):
        if joined[v]:
            succ[v] = (v + 1 + np.arange(sls)) % n
        else:
            i = int(np.searchsorted(old, v))
            succ[v] = old[(i + 1 + np.arange(sls)) % len(old)]
            pred[v] = old[(i - 1) % len(old)]
    nsucc = np.full(n, sls, dtype=np.uint8)
    ideal = OracleNet("chord", net.ids, net.xy).chord_fingers()
    fing = ideal.copy()
    # the old members' fingers point past the joined nodes: to the next old node
    for v in old:
        f = fing[v]
        bad = joined[f]
        f[bad] = old[pos[f[bad]] % len(old)]
    fing[joined] = NONE
    deque = np.full(n, 160, dtype=np.uint8)
    return net, joined, dict(pred=pred, succ=succ, nsucc=nsucc, fingers=fing, deque_size=deque)


def test_rounds_converge_to_the_stable_ring():
    n = 300
    net, joined, t = joined_ring(n, 0x57AB)
    o = OracleNet("chord", net.ids, net.xy, tables=t)
    ideal_fingers = OracleNet("chord", net.ids, net.xy).chord_fingers()
    for rnd in range(12):
        st = o.chord_stabilize()
        o.chord_fix_fingers()
        if st["lists_changed"] == 0 and st["pred_changed"] == 0:
            break
    pred, succ, nsucc = o.chord_lists()
    assert np.array_equal(pred, (np.arange(n) - 1) % n)
    assert np.array_equal(succ, (np.arange(n)[:, None] + 1 + np.arange(8)[None, :]) % n)
    assert (nsucc == 8).all()
    assert np.array_equal(o.chord_fingers(), ideal_fingers)
    assert rnd >= 1


def test_stabilize_round_counters():
    n = 300
    net, joined, t = joined_ring(n, 0x57AC)
    o = OracleNet("chord", net.ids, net.xy, tables=t)
    st = o.chord_stabilize()
    # round 1: a joined node notifies its successor, which takes it as predecessor; the old
    # predecessor learns of it only in round 2 (its successor's predecessor)
    assert st["pred_changed"] > 0 and st["succ_changed"] == 0
    st2 = o.chord_stabilize()
    assert st2["succ_changed"] > 0 and st2["lists_changed"] >= st2["succ_changed"]
