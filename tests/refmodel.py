"""Second, independent restatement of the reference semantics in pure Python.

Test infrastructure only.  Written separately from oracle/ovs_oracle.c (Python
ints instead of GMP-style limbs, a direct alpha = 1 loop instead of the event
list) so that the two restatements can check each other on small cases; the
reference itself cannot be built here.

Cites: OverlayKey.cc:587-644 (intervals), Chord.cc:422-674 (routing),
ChordFingerTable.cc:174-193, Chord.cc:845-875 (stable fingers),
IterativeLookup.cc:803-921,1067-1170 (alpha = 1 path), BaseOverlay.cc:1107-1146,
SimpleNodeEntry.cc:145-195 (delay).
"""
from __future__ import annotations

import bisect
import math

import numpy as np

M = 1 << 160


def to_int(w) -> int:
    return sum(int(w[i]) << (32 * i) for i in range(5))


# --- OverlayKey interval predicates -------------------------------------------
def between(x, a, b):
    if x == a:
        return False
    if a < b:
        return a < x < b
    return x > a or x < b


def between_r(x, a, b):
    if a == b and x == a:
        return True
    if a <= b:
        return a < x <= b
    return x > a or x <= b


def between_lr(x, a, b):
    if a == b and x == a:
        return True
    if a <= b:
        return a <= x <= b
    return x >= a or x <= b


# --- SimpleUnderlay delay -------------------------------------------------------
def simtime(d: float, rnd: bool) -> int:
    x = d * 1e9
    return math.floor(x + 0.5) if rnd else int(x)


def coord_ns(xy, a, b, rnd=True) -> int:
    dx = float(xy[a][0]) - float(xy[b][0])
    dy = float(xy[a][1]) - float(xy[b][1])
    s = dx * dx + dy * dy
    f = float(np.float32(math.sqrt(s)))
    return simtime(0.001 * f, rnd)


def msg_ns(nbytes: int, rnd=True, datarate=10e6) -> int:
    bw = simtime((nbytes * 8) / datarate, rnd)
    return 2 * bw  # tx serialisation + rx serialisation, access delay 0


# --- Chord ---------------------------------------------------------------------------
class ChordRing:
    def __init__(self, ids_words, xy, sls=8, rnd=True):
        self.ids = [to_int(w) for w in ids_words]
        assert all(self.ids[i] < self.ids[i + 1] for i in range(len(self.ids) - 1))
        self.n = len(self.ids)
        self.xy = xy
        self.ns = min(sls, self.n - 1)
        self.rnd = rnd
        self.fcache = {}

    def responsible(self, k):
        i = bisect.bisect_left(self.ids, k)
        return 0 if i == self.n else i

    def succ(self, c, j):
        return (c + 1 + j) % self.n

    def finger(self, c, pos):
        # getFinger(pos) of the converged table: trivial -> succ0
        me = self.ids[c]
        d = (self.ids[self.succ(c, 0)] - me) % M
        if (1 << pos) > d:
            return self.responsible((me + (1 << pos)) % M)
        return self.succ(c, 0)

    def decide(self, c, k):
        """-> (sibling_flag, next_node) of findNode(k, 1, 1) at node c."""
        me = self.ids[c]
        pred = self.ids[(c - 1) % self.n]
        if between_r(k, pred, me):
            return True, c
        s0 = self.succ(c, 0)
        if between_r(k, me, self.ids[s0]):
            return False, s0
        temp = None
        for j in range(self.ns - 1, -1, -1):
            if between_r(self.ids[self.succ(c, j)], me, k):
                temp = self.ids[self.succ(c, j)]
                break
        if temp is None:
            raise RuntimeError("Successor list broken")
        for pos in range(159, -1, -1):
            f = self.finger(c, pos)
            if between_lr(self.ids[f], temp, k):
                return False, f
        for j in range(self.ns - 1, -1, -1):
            sj = self.succ(c, j)
            if between(self.ids[sj], me, k):
                return False, sj
        raise RuntimeError("Error in Chord::closestPreceedingNode()")

    def lookup(self, kw, S, hop_max=50, call=83, resp=87, route=186, rpc_to=1.5, lk_to=10.0):
        k = to_int(kw)
        rnd = self.rnd
        sib, nxt = self.decide(S, k)
        if sib:
            return dict(responsible=S, hops=0, status=0, one_way_hops=0, latency_ns=0, hop_seq=[])
        t, hops, seq, visited = 0, 0, [], {S}
        cur = nxt
        while True:
            cd = coord_ns(self.xy, S, cur, rnd)
            rtt = msg_ns(call, rnd) + cd + msg_ns(resp, rnd) + cd
            if rtt >= simtime(rpc_to, rnd):
                st = 1 if t + simtime(rpc_to, rnd) > simtime(lk_to, rnd) else 2
                return dict(responsible=0xFFFFFFFF, hops=hops, status=st, one_way_hops=0, latency_ns=-1, hop_seq=seq)
            t += rtt
            if t > simtime(lk_to, rnd):
                return dict(responsible=0xFFFFFFFF, hops=hops, status=1, one_way_hops=0, latency_ns=-1, hop_seq=seq)
            hops += 1
            seq.append(cur)
            visited.add(cur)
            sib, nxt = self.decide(cur, k)
            if sib:
                R = cur
                lat = t + (msg_ns(route, rnd) + coord_ns(self.xy, S, R, rnd) if R != S else 0)
                return dict(responsible=R, hops=hops, status=0, one_way_hops=hops + (R != S), latency_ns=lat,
                            hop_seq=seq)
            if hop_max and hops >= hop_max:
                return dict(responsible=0xFFFFFFFF, hops=hops, status=3, one_way_hops=0, latency_ns=-1, hop_seq=seq)
            if nxt in visited:
                return dict(responsible=0xFFFFFFFF, hops=hops, status=4, one_way_hops=0, latency_ns=-1, hop_seq=seq)
            cur = nxt

    def lookup_call(self, kw, S, num_siblings=8, hop_max=50, call=83, resp=87, rpc_to=1.5, lk_to=10.0):
        """KBRTestApp LookupCall: the same iterative path; the responsible node answers
        [R, succ...] cut to num_siblings (a bigger FindNodeResponse: 61 B + 26 B per node), the
        response ends the lookup (no route message) and the siblings vector is that answer."""
        k = to_int(kw)
        rnd = self.rnd
        m = min(num_siblings, 1 + self.ns)
        resp_sib = 61 + 26 * m
        sib, nxt = self.decide(S, k)
        if sib:
            return dict(siblings=[(S + j) % self.n for j in range(m)], hops=0, status=0, latency_ns=0)
        t, hops, visited = 0, 0, {S}
        cur = nxt
        while True:
            sib, nxt = self.decide(cur, k)
            cd = coord_ns(self.xy, S, cur, rnd)
            rtt = msg_ns(call, rnd) + cd + msg_ns(resp_sib if sib else resp, rnd) + cd
            if rtt >= simtime(rpc_to, rnd):
                st = 1 if t + simtime(rpc_to, rnd) > simtime(lk_to, rnd) else 2
                return dict(siblings=[], hops=hops, status=st, latency_ns=-1)
            t += rtt
            if t > simtime(lk_to, rnd):
                return dict(siblings=[], hops=hops, status=1, latency_ns=-1)
            hops += 1
            visited.add(cur)
            if sib:
                return dict(siblings=[(cur + j) % self.n for j in range(m)], hops=hops, status=0, latency_ns=t)
            if hop_max and hops >= hop_max:
                return dict(siblings=[], hops=hops, status=3, latency_ns=-1)
            if nxt in visited:
                return dict(siblings=[], hops=hops, status=4, latency_ns=-1)
            cur = nxt

    def lookup_recursive(self, kw, S, hop_max=50, route=186):
        """Semi-recursive one-way route message: greedy forwarding S -> ... -> responsible,
        one UDP message of `route` bytes per hop (BaseOverlay.cc:1445-1582, 907-914)."""
        k = to_int(kw)
        cur, t, hops, seq = S, 0, 0, []
        while True:
            sib, nxt = self.decide(cur, k)
            if sib:
                return dict(responsible=cur, hops=hops, status=0, one_way_hops=hops, latency_ns=t, hop_seq=seq)
            if hops >= hop_max:
                return dict(responsible=0xFFFFFFFF, hops=0, status=3, one_way_hops=0, latency_ns=-1, hop_seq=seq)
            t += msg_ns(route, self.rnd) + coord_ns(self.xy, cur, nxt, self.rnd)
            hops += 1
            seq.append(nxt)
            cur = nxt


# --- Kademlia findNode (Kademlia.cc:357-382, 888-962, 1101-1246) on exported tables --
class KadTables:
    def __init__(self, ids_words, sib, bcount, bnodes, k=8, s=8):
        self.ids = [to_int(w) for w in ids_words]
        self.sib, self.bcount, self.bnodes = sib, bcount, bnodes
        self.k, self.s = k, s

    def _sorted_add(self, vec, cap, node, key):
        # BaseKeySortedVector::add with KeyXorMetric (NodeVector.h:432-512)
        d = self.ids[node] ^ key
        if len(vec) == cap and not d <= (self.ids[vec[-1]] ^ key):
            return -1
        for i, v in enumerate(vec):
            if self.ids[v] == self.ids[node]:
                return -1
            if d < (self.ids[v] ^ key):
                vec.insert(i, node)
                del vec[cap:]
                return i
        vec.append(node)          # only reached when not full
        return len(vec) - 1

    def bucket_index(self, c, key):
        d = key ^ self.ids[c]
        return d.bit_length() - 1 if d else -1

    def siblings(self, c):
        return [int(x) for x in self.sib[c] if x != 0xFFFFFFFF]

    def is_sibling_for(self, c, key, num_siblings=1):
        sib = self.siblings(c)
        if len(sib) < num_siblings:
            return True
        if len(sib) == 5 * self.s and (self.ids[c] ^ key) > (self.ids[c] ^ self.ids[sib[-1]]):
            return False
        res = []
        for x in sib:
            self._sorted_add(res, num_siblings, x, key)
        self._sorted_add(res, num_siblings, c, key)
        return any(self.ids[x] == self.ids[c] for x in res)

    def find_node(self, c, key, num_redundant=8, num_siblings=1):
        size = (num_siblings or 1) if self.is_sibling_for(c, key, num_siblings) else num_redundant
        res = []
        sib = self.siblings(c)
        if not sib:
            return [c]
        main = self.bucket_index(c, key)
        start = main
        end = self.bucket_index(c, self.ids[sib[-1]])

        def bucket(m):
            return [int(x) for x in self.bnodes[c][m][: self.bcount[c][m]]]

        if main != -1:
            for x in bucket(main):
                self._sorted_add(res, size, x, key)
        if start >= end or len(res) < size:
            for idx in range(start, end - 1, -1):
                if idx == main:
                    continue
                for x in bucket(idx):
                    self._sorted_add(res, size, x, key)
            for x in sib:
                self._sorted_add(res, size, x, key)
            self._sorted_add(res, size, c, key)
        idx = main + 1
        while len(res) < size and idx < 160:
            for x in bucket(idx):
                self._sorted_add(res, size, x, key)
            idx += 1
        return res
