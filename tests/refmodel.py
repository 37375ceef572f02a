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

    def lookup_call(self, kw, S, num_siblings=8, hop_max=50, call=83, resp=87, rpc_to=1.5, lk_to=10.0, resp_base=61):
        """KBRTestApp LookupCall: the same iterative path; the responsible node answers
        [R, succ...] cut to num_siblings (a bigger FindNodeResponse: 61 B + 26 B per node), the
        response ends the lookup (no route message) and the siblings vector is that answer."""
        k = to_int(kw)
        rnd = self.rnd
        m = min(num_siblings, 1 + self.ns)
        resp_sib = resp_base + 26 * m
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
class KoordeRing:
    """Second, independent reading of Koorde routing (src/overlay/koorde/Koorde.cc) on a converged
    ring, in Python integers: walks over the successor / de Bruijn lists are done by clockwise
    distance instead of the reference's interval loops, the de Bruijn pointer by bisection."""

    M = 1 << 160

    def __init__(self, ids_words, xy, sls=16, dbls=16, shift=4, use_other=True, use_suc=True, rnd=True):
        self.ids = [to_int(w) for w in ids_words]
        self.n = len(self.ids)
        self.xy = xy
        self.ns = min(sls, self.n - 1)
        self.dbls, self.shift, self.use_other, self.use_suc, self.rnd = dbls, shift, use_other, use_suc, rnd
        self.db = []          # (deBruijnNode, [deBruijnNodes])
        for v in range(self.n):
            self.db.append(self._debruijn(v))

    def d(self, a, b):
        """clockwise distance from key a to key b"""
        return (b - a) % self.M

    def succ(self, v, j):
        return (v + 1 + j) % self.n

    def responsible(self, k):
        i = bisect.bisect_left(self.ids, k)
        return 0 if i == self.n else i

    def _debruijn(self, v):
        """Koorde.cc:164-230 (+ the DeBruijnCall answer, 328-367) once the ring is stable"""
        M, me = self.M, self.ids[v]
        key = (me << self.shift) % M
        key = (key - (self.ids[self.succ(v, self.ns // 2)] - me)) % M
        pred = (v - 1) % self.n
        if 0 < self.d(me, key) <= self.d(me, self.ids[self.succ(v, 0)]):
            return v, [self.succ(v, j) for j in range(min(self.ns, self.dbls))]
        if 0 < self.d(self.ids[pred], key) <= self.d(self.ids[pred], me):
            return pred, [v] + [self.succ(v, j) for j in range(min(self.ns, self.dbls - 1))]
        R = self.responsible(key)
        return (R - 1) % self.n, [(R + j) % self.n for j in range(min(self.ns + 1, self.dbls))]

    def _walk(self, nodes, key):
        """the last of the clockwise-ordered `nodes` strictly before key, or nodes[-1] when key
        lies beyond them (walkSuccessorList / walkDeBruijnList)"""
        base = self.ids[nodes[0]]
        dk = self.d(base, key)
        if dk == 0 or dk > self.d(base, self.ids[nodes[-1]]):
            return nodes[-1]
        best = nodes[0]
        for x in nodes:
            if self.d(base, self.ids[x]) < dk:
                best = x
        return best

    def _start_key(self, v, dest):
        me, s0 = self.ids[v], self.ids[self.succ(v, 0)]
        nb = max(self.d(me, s0).bit_length() - 1, 0)
        while (160 - nb) % self.shift:
            nb -= 1
        key = (dest >> (160 - nb)) + ((me >> nb) << nb)
        key %= self.M
        for cand in (key, (key + (1 << nb)) % self.M):
            if 0 < self.d(me, cand) <= self.d(me, s0):
                return cand, nb + 1
        raise ValueError("invalid start key")

    def find_node(self, v, key, ext):
        """(next hop, ext) for Koorde::findNode at v; ext = [routeKey or None, step]; raises
        ValueError where the reference throws"""
        me, M = self.ids[v], self.M
        pred, s0 = (v - 1) % self.n, self.succ(v, 0)
        sl = [self.succ(v, j) for j in range(self.ns)]
        dbn, dbl = self.db[v]
        while True:
            if 0 < self.d(self.ids[pred], key) <= self.d(self.ids[pred], me) or key == me:
                return v, ext
            if 0 < self.d(me, key) <= self.d(me, self.ids[s0]):
                return s0, ext
            if self.use_other:
                t = self._walk(sl, key)
                if t != sl[-1]:
                    return t, ext
            brk = False
            if ext[0] is None:
                ext = list(self._start_key(v, key))
            rk, step = ext
            if 0 < self.d(me, rk) <= self.d(me, self.ids[s0]):
                if step > 160:
                    raise ValueError("bounding error")
                for i in range(self.shift):
                    pos = 160 - step - i
                    if pos < 0:
                        raise ValueError("bit position below 0")
                rk = ((rk << self.shift) % M) + ((key >> (160 - step - self.shift + 1)) & ((1 << self.shift) - 1))
                rk %= M
                ext = [rk, step + self.shift]
                if 0 < self.d(self.ids[dbn], rk) <= self.d(self.ids[dbn], self.ids[dbl[0]]):
                    h = dbn
                else:
                    h = self._walk(dbl, rk)
            else:
                brk = True
                if self.use_suc:
                    t = self._walk(sl, rk)
                    a, x = self.ids[t], self.ids[dbn]
                    # isBetween(x, a, rk): the open arc; a == rk is the whole ring but a
                    h = dbn if (x != a and (a == rk or self.d(a, x) < self.d(a, rk))) else t
                else:
                    h = s0
            if h != v or brk:
                return h, ext

    def lookup(self, kw, S, hop_max=50, call=104, resp=108, route=186, rpc_to=1.5, lk_to=10.0):
        """KBRTestApp one-way lookup, iterative, one path, one RPC in flight (Koorde's
        lookupRedundantNodes = lookupParallelRpcs = 1, merge off, visitOnlyOnce)"""
        k = to_int(kw)
        rnd = self.rnd
        pred = (S - 1) % self.n
        if 0 < self.d(self.ids[pred], k) <= self.d(self.ids[pred], self.ids[S]) or k == self.ids[S]:
            return dict(responsible=S, hops=0, status=0, one_way_hops=0, latency_ns=0, hop_seq=[])
        try:
            nxt, ext = self.find_node(S, k, [None, 1])
        except ValueError:
            return dict(responsible=0xFFFFFFFF, hops=0, status=5, one_way_hops=0, latency_ns=-1, hop_seq=[])
        t, hops, seq, visited = 0, 0, [], {S}
        if nxt in visited:
            return dict(responsible=0xFFFFFFFF, hops=0, status=4, one_way_hops=0, latency_ns=-1, hop_seq=seq)
        cur = nxt
        while True:
            try:
                nxt, ext2 = self.find_node(cur, k, list(ext))
            except ValueError:
                return dict(responsible=0xFFFFFFFF, hops=hops, status=5, one_way_hops=0, latency_ns=-1, hop_seq=seq)
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
            p = (cur - 1) % self.n
            if 0 < self.d(self.ids[p], k) <= self.d(self.ids[p], self.ids[cur]) or k == self.ids[cur]:
                R = cur
                lat = t + (msg_ns(route, rnd) + coord_ns(self.xy, S, R, rnd) if R != S else 0)
                return dict(responsible=R, hops=hops, status=0, one_way_hops=hops + (R != S), latency_ns=lat,
                            hop_seq=seq)
            if hop_max and hops >= hop_max:
                return dict(responsible=0xFFFFFFFF, hops=hops, status=3, one_way_hops=0, latency_ns=-1, hop_seq=seq)
            if nxt in visited:
                return dict(responsible=0xFFFFFFFF, hops=hops, status=4, one_way_hops=0, latency_ns=-1, hop_seq=seq)
            ext = ext2
            cur = nxt


def kad_num_buckets(b: int) -> int:
    """numBuckets = ((2^b) - 1) * (keylength / b) (Kademlia.cc:176)."""
    return ((1 << b) - 1) * (160 // b)


def kad_bucket_index(delta: int, b: int, first_on_layer: bool = False) -> int:
    """Kademlia::routingBucketIndex of a key whose XOR distance to the node is delta (357-382): the
    highest b-bit digit (positions 160-b, 160-2b, ... >= 0) that is not zero."""
    i = 160 - b
    while i >= 0 and (delta >> i) & ((1 << b) - 1) == 0:
        i -= b
    if i < 0:
        return -1
    per = (1 << b) - 1
    return (i // b) * per + (per - 1 if first_on_layer else ((delta >> i) & per) - 1)


def kad_bucket_size(index: int, k: int, bucket_type: int = 0, extra: int = 0) -> int:
    """Kademlia::routingBucketSize (384-411); 0 = unbounded (nkademlia)."""
    if bucket_type == 1:
        return 0
    if bucket_type == 2:
        import math
        limit = int(math.log(extra or 160) / math.log(2))
        off = limit - (160 - (index + 1))
        if off > 0 and 2 ** off > k:
            return 2 ** off
    return k


class KadTables:
    def __init__(self, ids_words, sib, bcount, bnodes, k=8, s=8, b=1, buckets=None):
        """buckets: per node a dict bucket index -> members (any b / size); else the k-stride
        bcount / bnodes arrays (b = 1)."""
        self.ids = [to_int(w) for w in ids_words]
        self.sib, self.bcount, self.bnodes = sib, bcount, bnodes
        self.k, self.s, self.b = k, s, b
        self.buckets = buckets

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

    def bucket_index(self, c, key, first=False):
        return kad_bucket_index(key ^ self.ids[c], self.b, first)

    def siblings(self, c):
        return [int(x) for x in self.sib[c] if x != 0xFFFFFFFF]

    def is_sibling_for(self, c, key, num_siblings=1):
        if num_siblings == 0:                      # exact-key lookups (Kademlia.cc:913-916)
            return self.ids[c] == key
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
        # numSiblings < 0: an exhaustive-iterative call, resultSize = numRedundantNodes (Kademlia.cc:1125-1127)
        if num_siblings < 0:
            size = num_redundant
        else:
            size = (num_siblings or 1) if self.is_sibling_for(c, key, num_siblings) else num_redundant
        res = []
        sib = self.siblings(c)
        if not sib:
            return [c]
        main = self.bucket_index(c, key)
        start = self.bucket_index(c, key, True)
        end = self.bucket_index(c, self.ids[sib[-1]])

        def bucket(m):
            if self.buckets is not None:
                return list(self.buckets[c].get(m, ()))
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
        while len(res) < size and idx < kad_num_buckets(self.b):
            for x in bucket(idx):
                self._sorted_add(res, size, x, key)
            idx += 1
        return res


# --- Kademlia iterative lookup as a discrete-event simulation --------------------------------
class KadLookupSim:
    """One KBRTestApp lookup over a Kademlia network, restated as OMNeT++ would run it: a future
    event set ordered by (arrival time, insertion order), every message hop a separate event --
    overlay -> UDP (zero delay), UDP -> UDP (SimpleNodeEntry::calcDelay with the sender's tx
    queue), UDP -> overlay (zero delay) -- the RPC timeout scheduled before the call is sent
    (BaseRpc.cc:256-271), the responder answering when its overlay handles the call
    (BaseOverlay::findNodeRpc, BaseOverlay.cc:1841-1915).  The lookup itself follows
    IterativeLookup / IterativePathLookup (IterativeLookup.cc:133-349, 406-449, 488-689,
    786-1195) with parallelPaths = 1, failedNodeRpcs = false, no verify / majority siblings.

    Independent of oracle/ovs_oracle.c, whose loop computes each response at send time and
    orders pending events by (time, insertion time, sequence); this one simulates the messages.
    findNode / isSiblingFor come from KadTables (another independent restatement)."""

    def __init__(self, tables: "KadTables", xy, redundant=8, alpha=3, merge=True, strict=True, visit_once=True,
                 accept_late_siblings=True, use_all=False, new_on_timeout=False, new_on_response=False,
                 finish_on_first_unchanged=False, hop_max=50, rnd=True, rpc_timeout=1.5, lookup_timeout=10.0,
                 datarate=10e6, k=8, call_bytes=83, resp_base=61, resp_node=26, route_bytes=186):
        self.T, self.xy = tables, xy
        self.cfg = dict(redundant=redundant, alpha=alpha, merge=merge, strict=strict, visit_once=visit_once,
                        late=accept_late_siblings, use_all=use_all, new_to=new_on_timeout,
                        new_resp=new_on_response, first_unch=finish_on_first_unchanged)
        self.hop_max, self.rnd, self.k = hop_max, rnd, k
        self.rpc_to, self.lk_to = simtime(rpc_timeout, rnd), simtime(lookup_timeout, rnd)
        self.datarate = datarate
        self.call_b, self.resp_b, self.resp_n, self.route_b = call_bytes, resp_base, resp_node, route_bytes

    # SimpleNodeEntry::calcDelay (SimpleNodeEntry.cc:155-195); SimpleUDP: 0 to itself (SimpleUDP.cc:322)
    def _delay(self, a, b, nbytes):
        if a == b:
            return 0
        bw = simtime(nbytes * 8 / self.datarate, self.rnd)
        fin = max(self.tx.get(a, 0), self.now) + bw
        self.tx[a] = fin
        return (fin - self.now) + coord_ns(self.xy, a, b, self.rnd) + bw

    def _schedule(self, t, kind, data):
        import heapq
        self.ins += 1
        heapq.heappush(self.fes, (t, self.ins, kind, data))

    def _dist(self, x):
        return self.T.ids[x] ^ self.key

    # LookupVector::add (BaseKeySortedVector::add, NodeVector.h:432-512), entries [node, alreadyUsed]
    def _nh_add(self, h):
        cap, nh = (2 * self.R if self.exh else self.R), self.nh
        if not self.cfg["merge"]:
            nh.append([h, False])
            return len(nh) - 1
        d = self._dist(h)
        if len(nh) == cap and not d <= self._dist(nh[-1][0]):
            return -1
        for i, e in enumerate(nh):
            if self.T.ids[e[0]] == self.T.ids[h]:
                return -1
            if d < self._dist(e[0]):
                nh.insert(i, [h, False])
                del nh[cap:]
                return i
        nh.append([h, False])
        return len(nh) - 1

    def _add_sibling(self, h):
        if len(self.siblings) < max(self.num_siblings, 1):       # parallelPaths 1: push_back if not full
            self.siblings.append(h)

    def _send_rpcs(self, num):
        """IterativePathLookup::sendRpc (IterativeLookup.cc:1067-1170)."""
        c = self.cfg
        if self.pfinished:
            return
        if self.hop_max and self.hops >= self.hop_max:
            self.pfinished, self.psuccess = True, False
            return
        if c["strict"]:
            num = min(num, c["alpha"] - self.pending)
        if num == 0 and self.pending == 0 and not c["first_unch"]:
            num = c["alpha"]
        i = 0
        while num > 0 and i < self.R:
            i += 1
            it = next((e for e in self.nh if not e[1] and e[0] not in self.dead), None)
            if it is None:
                break
            if not c["visit_once"] or it[0] not in self.visited:
                self.pending += 1
                num -= 1
                self._lookup_send(it[0], self.step)
            it[1] = True
        if self.pending == 0:
            if self.exh:   # exhaustive lookups always succeed: siblings = the first R next hops (1147-1156)
                for e in self.nh[: self.R]:
                    self._add_sibling(e[0])
                self.psuccess, self.pfinished = True, True
            else:
                self.psuccess, self.pfinished = False, True

    def _lookup_send(self, h, rpc_id):
        """IterativeLookup::sendRpc (656-689) + BaseRpc::sendRpcCall: timeout first, then the call."""
        if self.finished or not self.running:
            return
        if h not in self.rpcs:
            self.rpcs[h] = []
            self.nsent += 1
            self.live.add(h)
            self._schedule(self.now + self.rpc_to, "timeout", h)
            self._schedule(self.now, "call_udp", h)
            self.sent_at[h] = self.now
        self.rpcs[h].append(rpc_id)

    def _count_finished(self):
        if self.pfinished and not self.counted:
            self.counted = True
            self.finished_paths += 1
            self.min_hops = min(self.min_hops, self.hops)
            self.successful_paths += 1 if self.psuccess else 0

    def _path_timeout(self, dest=None):
        """IterativePathLookup::handleTimeout (935-1023), failedNodeRpcs = false."""
        if self.pfinished:
            return
        if self.exh and dest in self.dead:   # exhaustive: a dead node leaves nextHops (948-957)
            self.nh = [e for e in self.nh if e[0] != dest]
        self.pending -= 1
        if self.now > self.lk_to:
            self.pfinished, self.psuccess = True, False
            return
        if self.cfg["new_to"]:
            self._send_rpcs(1)
        elif self.pending == 0:
            self._send_rpcs(self.cfg["alpha"])

    def _path_response(self, src, closest, sib_flag):
        """IterativePathLookup::handleResponse (803-921)."""
        if self.pfinished:
            return
        if self.now > self.lk_to:
            self.pfinished, self.psuccess = True, False
            return
        if src != self.S:
            self.hops += 1
            self.hop_seq.append(src)
            self.rtts.append(self.now - self.sent_at[src])
            self.arrivals.append(self.now)
        self.visited.add(src)
        self.step += 1
        self.pending -= 1
        if closest and not self.cfg["merge"]:
            self.nh.clear()
        new = 0
        for h in closest:
            pos = self._nh_add(h)
            if 0 <= pos < self.R:
                new += 1
            if self.num_siblings == 0 and self.T.ids[h] == self.key:   # the key's node found (862-870)
                self.siblings = [h]
                self.pfinished, self.psuccess = True, True
                return
            if self.num_siblings and not self.exh and sib_flag:
                self._add_sibling(h)
        if not self.exh and sib_flag and closest and self.num_siblings:
            self.pfinished, self.psuccess = True, True
            return
        if new == 0 and self.cfg["new_resp"]:
            new = 1
        self._send_rpcs(min(new, self.cfg["alpha"]))

    def _check_stop(self):
        """IterativeLookup::checkStop (295-349), numSiblings > 0, retries = 0."""
        if (self.successful_paths >= 1 and self.num_siblings == 0 and self.siblings) or \
                (self.finished_paths == 1 and self.num_siblings > 0) or not self.rpcs:
            self.success |= self.psuccess or self.successful_paths >= 1
            self.running = False
            self.finished = True
            return True
        return False

    def run(self, key_words, S, num_siblings=1, lookup_call=False, exhaustive=0):
        """exhaustive = R > 0: an EXHAUSTIVE_ITERATIVE_ROUTING lookup with config.redundantNodes = R
        (Kademlia's bucket / sibling refresh with numSiblings = R, Kademlia.cc:1604-1611, 1658-1665;
        routingType = "exhaustive-iterative" lookups with R = lookupRedundantNodes)."""
        import heapq
        self.key = to_int(key_words)
        self.exh = exhaustive
        self.R = exhaustive if exhaustive else self.cfg["redundant"]
        self.sent_at, self.rtts, self.arrivals, self.calls = {}, [], [], []
        self.S, self.num_siblings = S, num_siblings
        self.fes, self.ins, self.now, self.tx = [], 0, 0, {}
        self.nh, self.visited, self.dead, self.rpcs, self.live = [], {S}, set(), {}, set()
        self.siblings, self.hop_seq = [], []
        self.hops = self.step = self.pending = 0
        self.pfinished = self.psuccess = self.counted = False
        self.finished, self.success, self.running = False, False, True
        self.finished_paths = self.successful_paths = 0
        self.min_hops, self.nsent = 1 << 30, 0
        T = self.T
        # IterativeLookup::start (133-244)
        nxt = T.find_node(S, self.key, self.k, -1 if self.exh else num_siblings)
        done = False
        if not nxt:
            self.finished, self.success, done = True, False, True
        elif num_siblings == 0 and T.ids[S] == self.key:     # exact-key lookup of the own key (171-184)
            self.siblings = [S]
            self.finished = self.success = done = True
        elif num_siblings and not self.exh and T.is_sibling_for(S, self.key, num_siblings):
            for h in nxt:
                self._add_sibling(h)
            self.finished = self.success = done = True
        if not done:
            for h in nxt:
                self._nh_add(h)
            self._send_rpcs(self.cfg["alpha"])
            done = self._check_stop()
        resp_of = {}
        while not done and self.fes:
            t, _, kind, h = heapq.heappop(self.fes)
            self.now = t
            if kind == "call_udp":            # source UDP: the call leaves through the tx queue
                ta = t + self._delay(S, h, self.call_b)
                self.calls.append((h, ta))
                self._schedule(ta, "call_app_at", h)
            elif kind == "call_app_at":       # responder UDP -> overlay (zero delay)
                self._schedule(t, "call_rpc", h)
            elif kind == "call_rpc":          # findNodeRpc at the responder
                # findNodeRpc: exhaustive calls ask findNode with numSiblings -1 and set no flag (1857-1871)
                res = T.find_node(h, self.key, self.R, -1 if self.exh else num_siblings)
                flag = False if self.exh else T.is_sibling_for(h, self.key, num_siblings)
                resp_of[h] = (res, flag)
                self._schedule(t, "resp_udp", h)
            elif kind == "resp_udp":          # responder UDP: response through its tx queue
                self._schedule(t + self._delay(h, S, self.resp_b + self.resp_n * len(resp_of[h][0])), "resp_app_at", h)
            elif kind == "resp_app_at":
                self._schedule(t, "resp_rpc", h)
            elif kind == "resp_rpc":          # BaseRpc: response before its timeout -> handleRpcResponse
                if h not in self.live:
                    continue
                self.live.discard(h)
                if self.finished or not self.running or h not in self.rpcs:
                    continue
                ids = self.rpcs.pop(h)
                res, flag = resp_of[h]
                handled = False
                for rid in ids:
                    if self.pfinished:
                        continue
                    acc = (self.cfg["use_all"] and self.cfg["merge"]) or rid == self.step
                    if not handled and (acc or self.exh or (flag and self.cfg["late"])):
                        self._path_response(h, res, flag)
                        handled = True
                    else:
                        self._path_timeout(h)
                    self._count_finished()
                done = self._check_stop()
            elif kind == "timeout":           # BaseRpc timeout -> handleRpcTimeout (588-654)
                if h not in self.live:
                    continue
                self.live.discard(h)
                if self.finished or not self.running or h not in self.rpcs:
                    continue
                ids = self.rpcs.pop(h)
                self.dead.add(h)
                for _ in ids:
                    if self.pfinished:
                        continue
                    self._path_timeout(h)
                    self._count_finished()
                done = self._check_stop()
        if not done:
            self._check_stop()
        # calls still leaving the source's UDP when the lookup ended reach their destination anyway
        # (IterativeLookup::stop cancels the RPC state, not the message; IterativeLookup.cc:256-261)
        now_end = self.now
        for t, _, kind, h in sorted(self.fes):
            if kind == "call_udp":
                self.now = t
                self.calls.append((h, t + self._delay(S, h, self.call_b)))
        self.now = now_end
        valid = self.success and self.finished
        hops = 0 if self.min_hops == 1 << 30 else self.min_hops
        if lookup_call:
            return dict(siblings=list(self.siblings) if valid else [], hops=hops, status=self._status(valid),
                        is_valid=int(valid), latency_ns=self.now if valid else -1, rpcs=self.nsent,
                        responders=list(self.hop_seq), rtt_ns=list(self.rtts), tarr_ns=list(self.arrivals),
                        calls=list(self.calls))
        if not valid or not self.siblings:
            return dict(responsible=0xFFFFFFFF, hops=hops, status=self._status(False), one_way_hops=0,
                        latency_ns=-1, hop_seq=self.hop_seq, rpcs=self.nsent)
        R = self.siblings[0]
        # SendToKeyListener::lookupFinished -> sendRouteMessage (BaseOverlay.cc:1107-1146, 1241-1259)
        lat = self.now + self._delay(S, R, self.route_b)
        return dict(responsible=R, hops=hops, status=0, one_way_hops=hops + (R != S), latency_ns=lat,
                    hop_seq=self.hop_seq, rpcs=self.nsent)

    def _status(self, valid):
        if valid:
            return 0
        if self.now > self.lk_to:
            return 1
        if self.dead:
            return 2
        if self.hop_max and self.hops >= self.hop_max:
            return 3
        return 4


# --- Kademlia maintenance: routingAdd and a synchronous refresh round -------------------------
class KadMaint:
    """A network's Kademlia tables as a running OverSim node keeps them, written from the reference
    independently of oracle/ovs_oracle.c: per node the sibling table as a Python list kept sorted by
    XOR distance to the node (KademliaBucket with its comparator, Kademlia.cc:179, 315-317) and the
    routing buckets as a dict bucket index -> list in LRU order (push_back / erase, 432-756)."""

    def __init__(self, ids_words, sib, bcount=None, bnodes=None, k=8, s=8, b=1, bucket_type=0, node_limit=1000,
                 extra=0, bucket_off=None, bucket_nodes=None):
        """k-stride bcount / bnodes (b = 1) or CSR bucket_off / bucket_nodes (any b)."""
        self.ids = [to_int(w) for w in ids_words]
        self.ids_words = ids_words
        self.k, self.s, self.b = k, s, b
        self.bucket_type, self.node_limit, self.extra = bucket_type, node_limit, extra
        self.nb = kad_num_buckets(b)
        n = len(self.ids)
        self.sib = []
        self.bk = []
        for v in range(n):
            mine = [int(x) for x in sib[v] if x != 0xFFFFFFFF]
            self.sib.append(sorted(mine, key=lambda x: self.ids[x] ^ self.ids[v]))
            if bucket_off is not None:
                row = {}
                for m in range(self.nb):
                    o0, o1 = int(bucket_off[v * self.nb + m]), int(bucket_off[v * self.nb + m + 1])
                    if o1 > o0:
                        row[m] = [int(x) for x in bucket_nodes[o0:o1]]
                self.bk.append(row)
            else:
                self.bk.append({m: [int(x) for x in bnodes[v][m][: bcount[v][m]]] for m in range(160) if bcount[v][m]})
        self.rts = [sum(len(x) for x in row.values()) for row in self.bk]   # currentRoutingTableSize

    def arrays(self):
        n, S5 = len(self.ids), 5 * self.s
        sib = [[0xFFFFFFFF] * S5 for _ in range(n)]
        cnt = [[0] * 160 for _ in range(n)]
        nodes = [[[0xFFFFFFFF] * self.k for _ in range(160)] for _ in range(n)]
        for v in range(n):
            for i, x in enumerate(self.sib[v]):
                sib[v][i] = x
            for m, lst in self.bk[v].items():
                cnt[v][m] = len(lst)
                for j, x in enumerate(lst):
                    nodes[v][m][j] = x
        return sib, cnt, nodes

    def csr(self):
        """(siblings rows, bucket_off, bucket_nodes) as orc_kad_export_csr lays them out."""
        S5 = 5 * self.s
        sib = [list(x) + [0xFFFFFFFF] * (S5 - len(x)) for x in self.sib]
        off, nodes = [0], []
        for row in self.bk:
            for m in range(self.nb):
                nodes += row.get(m, [])
                off.append(len(nodes))
        return sib, off, nodes

    def routing_add(self, v, h, alive):
        """Kademlia::routingAdd (Kademlia.cc:432-756): secureMaintenance, pingNewSiblings, activePing
        and proximityNeighborSelection off; every bucketType (routingBucketSize 384-411, the nkademlia
        branch 620-664).  Returns its result."""
        if h == v:
            return False
        me = self.ids[v]
        sib = self.sib[v]
        if h in sib:
            return True
        b = kad_bucket_index(self.ids[h] ^ me, self.b)
        bucket = self.bk[v].get(b)
        if bucket is not None and h in bucket:
            if alive:
                bucket.remove(h)
                bucket.append(h)
            return True
        cap = 5 * self.s
        d = self.ids[h] ^ me
        result = False
        if len(sib) < cap or d <= (self.ids[sib[-1]] ^ me):      # siblingTable->isAddable
            pos = next((i for i, x in enumerate(sib) if d < (self.ids[x] ^ me)), len(sib))
            sib.insert(pos, h)
            if len(sib) <= cap:
                return True
            h = sib.pop()                                        # preempted: goes to its bucket
            result = True
        b = kad_bucket_index(self.ids[h] ^ me, self.b)
        assert b >= 0, "bucket index -1: the reference dereferences a NULL bucket"
        bucket = self.bk[v].setdefault(b, [])
        if self.bucket_type == 1:                 # nkademlia (620-664): a global table limit
            if len(bucket) >= self.k and self.rts[v] >= self.node_limit:
                return False
            bucket.append(h)
            self.rts[v] += 1
            return True
        if len(bucket) < kad_bucket_size(b, self.k, self.bucket_type, self.extra):
            bucket.append(h)
            self.rts[v] += 1
            return True
        return result

    def refresh_keys(self, v):
        """handleBucketRefreshTimerExpired's bucket keys (Kademlia.cc:1631-1676): self ^ ((d+1) << i)
        for the digits i = 160-b .. diff and d = 0 .. 2^b-2, diff = 160 - b*(shared digits + 1)."""
        if not self.sib[v]:
            return []
        me = self.ids[v]
        front = self.ids[self.sib[v][0]] ^ me
        shared_bits = 160 - front.bit_length()
        diff = 160 - self.b * (shared_bits // self.b + 1)
        out = []
        for i in range(160 - self.b, diff - 1, -self.b):
            for d in range((1 << self.b) - 1):
                out.append(me ^ ((d + 1) << i))
        return out

    def round(self, xy, nodes, flags, lookup_cfg, R_bucket=8):
        """One synchronous maintenance round: the listed nodes' exhaustive refresh lookups on the
        round-start tables (KadLookupSim), then at every node the routingAdds of the calls that reached
        it and of its handled responses (carried nodes not alive, then the responder alive), in
        simulated-time order with ties (calls first, task, index)."""
        T = KadTables.__new__(KadTables)            # the round-start tables, as findNode reads them
        T.ids, T.k, T.s, T.b = self.ids, self.k, self.s, self.b
        T.sib = [list(x) + [0xFFFFFFFF] * (5 * self.s - len(x)) for x in self.sib]
        T.buckets = [{m: list(l) for m, l in row.items()} for row in self.bk]
        T.bcount = T.bnodes = None
        sim = KadLookupSim(T, xy, k=self.k, **lookup_cfg)
        tasks = []
        for v, f in zip(nodes, flags):
            if f & 1:
                tasks.append((v, self.ids[v], 5 * self.s))
            if f & 2:
                tasks += [(v, key, R_bucket) for key in self.refresh_keys(v)]
        events = {}
        for t, (v, key, R) in enumerate(tasks):
            words = [(key >> (32 * i)) & 0xFFFFFFFF for i in range(5)]
            m = sim.run(words, v, num_siblings=R, lookup_call=True, exhaustive=R)
            for i, (x, tc) in enumerate(m["calls"]):
                events.setdefault(x, []).append((tc, 0, t, i, v, None))
            for i, (x, ta) in enumerate(zip(m["responders"], m["tarr_ns"])):
                events.setdefault(v, []).append((ta, 1, t, i, x, T.find_node(x, key, R, -1)))
        for v, ev in events.items():
            for _, kind, _, _, x, carried in sorted(ev, key=lambda e: e[:4]):
                if kind == 0:
                    self.routing_add(v, x, True)
                else:
                    for c in carried:
                        self.routing_add(v, c, False)
                    self.routing_add(v, x, True)
        return len(tasks)


# --- EpiChord::findNode on one routing snapshot ---------------------------------
def epichord_find_node(keys, self_i, succ, pred, full_bits, list_size, cache, key, src, now, cache_ttl, R):
    """EpiChord.cc:517-629 served by node self_i, written from the reference independently of
    oracle/ovs_oracle_epichord.c: Python ints, the finger cache as a dict node -> [lastUpdate, ttl],
    the node lists as plain Python lists ordered by ring offset, and findBestHops as a walk over the
    live nodes sorted by clockwise distance from self + 1 (EpiChordFingerCache.cc:309-356).

    keys: list of int node keys; succ / pred: node indices closest first; full_bits: bit 0 / 1 =
    successorList / predecessorList->isFull(); cache: {node: (lastUpdate, ttl)}; src None = a local
    call.  Returns (status, [(node, lastUpdate)]): status 0 ok, -1 the reference throws, -2 it
    dereferences an empty cache."""
    me = keys[self_i]
    cache = {x: [lu, ttl] for x, (lu, ttl) in cache.items()}

    def off_fwd(x):      # succ map key + 1
        return (keys[x] - me) % M

    def off_bwd(x):
        return (me - keys[x]) % M

    # nodeMaps: real entries, plus thisNode (offset 0 -> key M - 1, the largest) when not full
    lists = {"succ": [list(succ), not (full_bits & 1), off_fwd], "pred": [list(pred), not (full_bits & 2), off_bwd]}

    def upd(x, lu, ttl):                 # EpiChordFingerCache::updateFinger 79-127
        if x is None or x == self_i:
            return
        if x in cache:
            e = cache[x]
            e[0] = max(e[0], lu)
            if e[1] > 0 and (ttl > e[1] or ttl == 0):
                e[1] = ttl
        else:
            cache[x] = [lu, ttl]

    def last_of(name):                   # getNode(getSize() - 1)
        ent, has_self, _ = lists[name]
        return self_i if has_self else ent[-1]

    def add(name, x):                    # EpiChordNodeList::addNode(x, resize = true) 108-161
        ent, has_self, off = lists[name]
        if x not in ent:
            ent.append(x)
            ent.sort(key=off)
        upd(x, now, 0)
        if len(ent) + (1 if has_self else 0) > list_size:
            if has_self:                 # thisNode has the largest offset: it goes first
                lists[name][1] = False
            else:
                gone = ent.pop()
                if gone in cache:        # setFingerTTL(gone) with the cache's ttl
                    cache[gone][1] = cache_ttl

    excl = {self_i}
    if src is not None:
        excl.add(src)
        upd(src, now, cache_ttl)         # receiveNewNode 1178-1209, direct
        for name, inside in (("succ", lambda x: between(keys[x], me, keys[last_of("succ")])),
                             ("pred", lambda x: between(keys[x], keys[last_of("pred")], me))):
            ent, has_self, _ = lists[name]
            contains = src in ent or (has_self and src == self_i)
            if not contains and (has_self or inside(src)):
                add(name, src)
    s_ent, p_ent = lists["succ"][0], lists["pred"][0]
    succ0 = s_ent[0] if s_ent else self_i
    pred0 = p_ent[0] if p_ent else self_i
    out = []
    if not p_ent:
        sib = (not s_ent) or key == me
    else:
        sib = between_r(key, keys[pred0], me)
    if sib:
        out.append((self_i, now))
        if p_ent:
            out.append((pred0, cache[pred0][0] if pred0 in cache else now))
        if s_ent:
            out.append((succ0, cache[succ0][0] if succ0 in cache else now))
        return 0, out
    if src is None:
        def rd(a, b):
            return min((a - b) % M, (b - a) % M)
        choice = pred0 if rd(keys[pred0], key) < rd(keys[succ0], key) else succ0
    elif between(me, keys[src], key):
        choice = succ0
    else:
        choice = pred0
    if choice in cache:
        out.append((choice, cache[choice][0]))
        excl.add(choice)
    live = sorted((x for x, (lu, ttl) in cache.items() if not (ttl > 0 and lu + ttl < now)),
                  key=lambda x: (keys[x] - me - 1) % M)
    if not live:
        return -2, out
    target = (key - me - 1) % M
    pos = next((i for i, x in enumerate(live) if (keys[x] - me - 1) % M >= target), 0)
    # forward to the first live node not excluded (at most once round the ring)
    for step in range(len(live)):
        j = (pos + step) % len(live)
        if live[j] not in excl:
            break
    else:
        return (0 if out else -1), out
    # then backwards from it, R nodes not excluded, at most once round
    taken = 0
    for step in range(len(live)):
        x = live[(j - step) % len(live)]
        if taken >= R:
            break
        if x not in excl:
            out.append((x, cache[x][0]))
            taken += 1
    return (0 if out else -1), out


# --- recursive routing over Kademlia tables (R/Kademlia) -------------------------------------
class KadRecursiveSim:
    """Recursive (semi / full) routing of one message over Kademlia tables, read from
    BaseOverlay::sendToKey / handleBaseOverlayMessage (BaseOverlay.cc:880-1004, 1380-1582) and
    Kademlia::recursiveRoutingHook (Kademlia.cc:1022-1057, altRecMode off): a route message carries
    its source and last hop; every node it reaches other than its source first sends a
    KademliaRoutingInfoMessage (findNode(key, k, s) nodes, 47 + 27 n + 28 B) to the source, which
    occupies the node's tx queue ahead of whatever the node sends next.  LookupCalls go through
    RecursiveLookup (RecursiveLookup.cc:52-139): a routed FindNodeCall, answered by findNodeRpc at
    the delivering node, the response sent back by UDP (semi) or routed to the source's key
    (full).  Independent of the oracle's rec_route; findNode / isSiblingFor from KadTables."""

    ROUTE_HDR = 53          # BASEROUTE_L 424 bits
    CALL = 55               # FINDNODECALL_L 440 bits

    def __init__(self, tables: "KadTables", xy, k=8, s=8, rec_redundant=3, redundant=8, hop_max=50, rnd=True,
                 datarate=10e6, route_bytes=186, resp_base=61, resp_node=26, key_timeout=10.0):
        self.T, self.xy, self.k, self.s = tables, xy, k, s
        self.recR, self.R, self.hop_max, self.rnd, self.datarate = rec_redundant, redundant, hop_max, rnd, datarate
        self.route_b, self.resp_b, self.resp_n = route_bytes, resp_base, resp_node
        self.key_to = simtime(key_timeout, rnd)

    def _send(self, q, a, b, nbytes, now):
        """SimpleNodeEntry::calcDelay with node a's queue q[a]; the arrival time at b."""
        if a == b:
            return now
        bw = simtime(nbytes * 8 / self.datarate, self.rnd)
        fin = max(q.get(a, 0), now) + bw
        q[a] = fin
        return fin + coord_ns(self.xy, a, b, self.rnd) + bw

    def _info(self, x, key):
        return 47 + 27 * len(self.T.find_node(x, key, self.k, self.s)) + 28

    def walk(self, key, src, ns_src, nbytes, now=0, q=None, source_routing=False):
        """(delivered node or None, hops, time, status, queues, hop list).  source_routing: the
        message records its senders (visitedHops, BaseOverlay.cc:888-897) and the forwarding nodes
        skip them too (1502-1516); its length stays the one set at creation (1398)."""
        q = {} if q is None else q
        msg = dict(src=src, last=src, hops=0, visited=[])
        node, t, path = src, now, []
        self.visited = msg["visited"]
        while True:
            ns = ns_src if node == src else 1
            if node != src:
                if source_routing:
                    msg["visited"].append(msg["last"])
                q.pop(node, None)                      # the queue is idle when the message arrives
                if self.T.is_sibling_for(node, key, 1):
                    self._send(q, node, src, self._info(node, key), t)   # the hook, then delivery
                    return node, msg["hops"], t, 0, q, path
            hops = self.T.find_node(node, key, self.recR, ns)
            if not hops:
                return None, 0, t, 4, q, path
            if msg["hops"] >= self.hop_max:
                return None, 0, t, 3, q, path
            sib = self.T.is_sibling_for(node, key, ns)
            nxt = None
            for h in hops:
                if (h == msg["last"] and h != node) or (h == src and node != src) or (h == node and not sib):
                    continue
                if h in msg["visited"]:
                    continue
                nxt = h
                break
            if nxt is None:
                return None, 0, t, 4, q, path
            if nxt == node:
                return node, msg["hops"], t, 0, q, path
            if node != src:
                self._send(q, node, src, self._info(node, key), t)
            t = self._send(q, node, nxt, nbytes, t)
            msg["hops"] += 1
            msg["last"] = node
            path.append(nxt)
            node = nxt

    def route(self, key, src, source_routing=False):
        key = to_int(key) if not isinstance(key, int) else key
        d, hops, t, st, _, path = self.walk(key, src, 1, self.route_b, source_routing=source_routing)
        if st:
            return dict(responsible=0xFFFFFFFF, hops=0, status=st, latency_ns=-1, hop_seq=path)
        return dict(responsible=d, hops=hops, status=0, latency_ns=t, hop_seq=path)

    def lookup_call(self, key, src, ns, full=False, source_routing=False):
        key = to_int(key) if not isinstance(key, int) else key
        d, _, t, st, q, _ = self.walk(key, src, ns, self.ROUTE_HDR + self.CALL + 28, source_routing=source_routing)
        visited = list(self.visited)
        fail = dict(num_siblings=0, hops=0, is_valid=0, latency_ns=-1, siblings=[])
        if st:
            return dict(fail, status=st)
        res = self.T.find_node(d, key, self.R, ns)
        flag = self.T.is_sibling_for(d, key, ns)
        if d != src:
            nbytes = self.resp_b + self.resp_n * len(res)
            if source_routing:
                # BaseRpc::internalSendRpcResponse (BaseRpc.cc:575-588): back along the visited hops,
                # last first; every node but the response's source (d) runs the hook toward d first
                skey = self.T.ids[src]
                node = d
                for nxt in reversed(visited):
                    if node != d:
                        q.pop(node, None)
                        self._send(q, node, d, self._info(node, skey), t)
                    t = self._send(q, node, nxt, self.ROUTE_HDR + nbytes, t)
                    node = nxt
            elif not full:
                t = self._send(q, d, src, nbytes, t)
            else:
                back, _, t, st2, _, _ = self.walk(self.T.ids[src], d, 1, self.ROUTE_HDR + nbytes, t, {d: q.get(d, 0)})
                if st2 or back != src:
                    return dict(fail, status=2)
        if t >= 2 * self.key_to:
            return dict(fail, status=2)
        if not flag or not res:
            return dict(fail, status=6)
        return dict(num_siblings=len(res), hops=0, status=0, is_valid=1, latency_ns=t, siblings=list(res))
