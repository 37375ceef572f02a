"""EpiChord routing snapshots and FindNodeCalls for the parity tests (test infrastructure only).

A snapshot is what EpiChord::findNode reads at a node (EpiChord.cc:517-629): its successor and
predecessor lists (EpiChordNodeList: closest first, isFull()), and its live finger cache
(EpiChordFingerCache::liveCache: node, lastUpdate, ttl).  The generator draws them the way a running
network leaves them: list members are cached with ttl 0 (EpiChordNodeList::addNode sets it,
EpiChordNodeList.cc:141-143), other entries carry cacheTTL and lastUpdates spread over the past, some
already expired; a share of the nodes has short lists (a freshly joined node, or a list that lost a
member), a few have stale list members, empty caches, or lists that miss their true neighbours.
"""
from __future__ import annotations

import numpy as np

from oversim_amd import workload as W

NONE = 0xFFFFFFFF
SEC = 1_000_000_000


def make_snapshot(n: int, seed: int, list_size: int = 4, cache_per_node: int = 12, cache_ttl_s: float = 120.0,
                  now_ns: int = 500 * SEC):
    rng = np.random.default_rng(seed)
    ids = W.sorted_unique_ids(n, seed)
    L = list_size
    succ = np.full((n, L), NONE, dtype=np.uint32)
    pred = np.full((n, L), NONE, dtype=np.uint32)
    nsucc = np.zeros(n, dtype=np.uint8)
    npred = np.zeros(n, dtype=np.uint8)
    full = np.zeros(n, dtype=np.uint8)
    ttl = int(cache_ttl_s * SEC)
    offs, nodes, lasts, ttls = [0], [], [], []
    for v in range(n):
        kind = rng.random()
        # successor / predecessor lists: the true neighbours, sometimes short or skipping a node
        for side, arr, cnt, bit in ((1, succ, nsucc, 1), (-1, pred, npred, 2)):
            want = min(L, n - 1)
            if kind < 0.15:
                want = int(rng.integers(0, want + 1))
            step_skip = 1 + (rng.random() < 0.1)
            ent = []
            j = v
            while len(ent) < want:
                j = (j + side * (step_skip if not ent else 1)) % n
                if j == v or j in ent:
                    break
                ent.append(j)
            arr[v, :len(ent)] = ent
            cnt[v] = len(ent)
            # isFull: a full list, or (rarely) a full list that lost a member (thisNode not back in it)
            if len(ent) == L or (0 < len(ent) < L and rng.random() < 0.2 and kind < 0.15):
                full[v] |= bit
        # finger cache: the list members (ttl 0) and random other nodes
        members = set(succ[v, :nsucc[v]].tolist()) | set(pred[v, :npred[v]].tolist())
        k = 0 if rng.random() < 0.03 else int(rng.integers(0, cache_per_node + 1))
        others = set(rng.integers(0, n, size=k).tolist()) - {v} - members
        ent = []
        for x in sorted(members):
            if rng.random() < 0.9:
                ent.append((x, int(rng.integers(now_ns - 200 * SEC, now_ns + 1)), 0 if rng.random() < 0.8 else ttl))
        for x in sorted(others):
            ent.append((x, int(rng.integers(now_ns - 3 * ttl, now_ns + 1)), ttl if rng.random() < 0.9 else 0))
        rng.shuffle(ent)
        for x, lu, t in ent:
            nodes.append(x); lasts.append(lu); ttls.append(t)
        offs.append(len(nodes))
    return dict(ids=ids, n=n, L=L, succ=succ, nsucc=nsucc, pred=pred, npred=npred, full=full,
                cache_off=np.array(offs, dtype=np.uint64), cache_node=np.array(nodes, dtype=np.uint32),
                cache_last=np.array(lasts, dtype=np.int64), cache_ttl=np.array(ttls, dtype=np.int64),
                cache_ttl_param=ttl, now=now_ns)


def make_queries(snap: dict, m: int, seed: int):
    """FindNodeCalls: responder, key (random keys, node IDs, keys next to the responder), source (a
    random node, a list member, the responder's neighbours, or a local call), simulated time."""
    rng = np.random.default_rng(seed)
    n, ids = snap["n"], snap["ids"]
    node = rng.integers(0, n, size=m).astype(np.uint32)
    keys = W.random_keys(m, rng)
    sel = rng.random(m)
    nid = rng.integers(0, n, size=m)
    keys[sel < 0.3] = ids[nid[sel < 0.3]]
    near = (sel >= 0.3) & (sel < 0.4)
    keys[near] = ids[(node[near].astype(np.int64) + rng.integers(-2, 3, size=near.sum())) % n]
    src = rng.integers(0, n, size=m).astype(np.uint32)
    s2 = rng.random(m)
    nb = (s2 < 0.25)
    src[nb] = ((node[nb].astype(np.int64) + rng.choice([-3, -2, -1, 1, 2, 3, 5], size=nb.sum())) % n).astype(np.uint32)
    src[s2 > 0.92] = NONE
    now = snap["now"] + rng.integers(-50 * SEC, 100 * SEC, size=m).astype(np.int64)
    return node, keys, src, now
