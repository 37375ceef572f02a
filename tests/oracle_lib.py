"""ctypes binding of the CPU oracle (oracle/ovs_oracle.h) -- test infrastructure only.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this.
"""
from __future__ import annotations

import ctypes as C
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
_SO = ROOT / "oracle" / "_build" / "libovs_oracle.so"

ORC_FAIL = 0xFFFFFFFFFFFFFFFF

ROUTE_DTYPE = np.dtype([("responsible", "<u4"), ("hops", "<u2"), ("status", "u1"),
                        ("one_way_hops", "u1"), ("latency_ns", "<i8")])

LOOKUP_DTYPE = np.dtype([("num_siblings", "<u4"), ("hops", "<u2"), ("status", "u1"),
                         ("is_valid", "u1"), ("latency_ns", "<i8")])


class OrcParams(C.Structure):
    _fields_ = [
        ("hopCountMax", C.c_int32), ("successorListSize", C.c_int32), ("numFingerCandidates", C.c_int32),
        ("k", C.c_int32), ("s", C.c_int32), ("b", C.c_int32),
        ("lookupRedundantNodes", C.c_int32), ("lookupParallelRpcs", C.c_int32), ("lookupMerge", C.c_int32),
        ("lookupStrictParallelRpcs", C.c_int32), ("lookupVisitOnlyOnce", C.c_int32),
        ("lookupAcceptLateSiblings", C.c_int32), ("lookupUseAllParallelResponses", C.c_int32),
        ("lookupNewRpcOnEveryTimeout", C.c_int32), ("lookupNewRpcOnEveryResponse", C.c_int32),
        ("lookupFinishOnFirstUnchanged", C.c_int32), ("numSiblings", C.c_int32), ("simtimeRound", C.c_int32),
        ("rpcUdpTimeout", C.c_double), ("lookupTimeout", C.c_double), ("datarate", C.c_double),
        ("accessDelay", C.c_double), ("callBytes", C.c_int32), ("respBaseBytes", C.c_int32),
        ("respPerNodeBytes", C.c_int32), ("routeBytes", C.c_int32), ("kadSeed", C.c_uint64),
        ("routingType", C.c_int32), ("recNumRedundantNodes", C.c_int32),
        ("shiftingBits", C.c_int32), ("deBruijnListSize", C.c_int32), ("useOtherLookup", C.c_int32),
        ("useSucList", C.c_int32),
        ("bucketType", C.c_int32), ("globalNodeLimit", C.c_int32), ("extraNodesFinalBucket", C.c_int32),
        ("rpcKeyTimeout", C.c_double), ("extendedFingerTable", C.c_int32), ("measureAuthBlock", C.c_int32),
    ]

    def replace(self, **kw) -> "OrcParams":
        p = OrcParams()
        C.memmove(C.byref(p), C.byref(self), C.sizeof(OrcParams))
        for k, v in kw.items():
            setattr(p, k, v)
        return p


_L = None


def lib() -> C.CDLL:
    global _L
    if _L is None:
        if not _SO.exists():
            import subprocess
            subprocess.run(["make", "-s", "-C", str(ROOT / "oracle")], check=True)
        L = C.CDLL(str(_SO))
        vp, u32, u64, i32 = C.c_void_p, C.c_uint32, C.c_uint64, C.c_int32
        for name, args, res in [
            ("orc_key_cmp", [vp, vp], C.c_int),
            ("orc_key_add", [vp, vp, vp], None),
            ("orc_key_sub", [vp, vp, vp], None),
            ("orc_key_xor", [vp, vp, vp], None),
            ("orc_key_between", [C.c_int, vp, vp, vp, C.c_int], C.c_int),
            ("orc_key_bit_range", [vp, u32, u32], u32),
            ("orc_key_shared_prefix", [vp, vp, u32], u32),
            ("orc_key_log2", [vp], C.c_int),
            ("orc_key_pow2", [u32, vp], None),
            ("orc_params_chord_default", [vp], None),
            ("orc_params_kad_default", [vp], None),
            ("orc_params_koorde_default", [vp], None),
            ("orc_koorde_build", [vp, u32, vp, vp], vp),
            ("orc_koorde_export", [vp, vp, vp, vp], None),
            ("orc_koorde_find_node", [vp, u32, vp, vp, C.POINTER(C.c_int), C.POINTER(C.c_int)], u32),
            ("orc_chord_build", [vp, u32, vp, vp], vp),
            ("orc_chord_build_tables", [vp, u32, vp, vp, vp, vp, u32, vp, vp, vp], vp),
            ("orc_kad_build", [vp, u32, vp, vp], vp),
            ("orc_chord_build_lazy", [vp, u32, vp, vp], vp),
            ("orc_kad_build_lazy", [vp, u32, vp, vp], vp),
            ("orc_kad_build_tables", [vp, u32, vp, vp, vp, vp, vp], vp),
            ("orc_cap_failed", [], C.c_int),
            ("orc_clear_error", [], None),
            ("orc_net_free", [vp], None),
            ("orc_kad_export", [vp, vp, vp, vp], None),
            ("orc_chord_export_fingers", [vp, vp], None),
            ("orc_find_node", [vp, u32, vp, C.c_int, C.c_int, vp, C.POINTER(C.c_int)], C.c_int),
            ("orc_route_batch", [vp, vp, vp, u64, vp, vp, vp, C.c_int], u64),
            ("orc_delay_ns", [vp, u32, u32, i32], C.c_int64),
            ("orc_coord_dist", [vp, u32, u32], C.c_float),
            ("orc_last_error", [], C.c_char_p),
            ("orc_kbrtest_stats", [vp, vp, vp, vp, u64, C.c_double, C.c_int, i32, vp], None),
            ("orc_chord_fix_fingers", [vp, vp, u64, C.POINTER(u64), C.POINTER(u64), C.c_int], u64),
            ("orc_lookup_batch", [vp, vp, vp, u64, C.c_int, vp, vp, C.c_int], C.c_int),
            ("orc_chord_stabilize", [vp, vp, u64, C.POINTER(u64), C.POINTER(u64)], u64),
            ("orc_chord_export_lists", [vp, vp, vp, vp], None),
            ("orc_kad_exhaustive_batch", [vp, vp, vp, u64, C.c_int, vp, vp, vp, vp, vp, C.c_int], C.c_int),
            ("orc_kad_refresh_keys", [vp, vp, u64, vp, vp, vp, u64], u64),
            ("orc_kad_exhaustive_batch_t", [vp, vp, vp, u64, C.c_int, vp, vp, vp, vp, vp, vp, vp, C.c_int, vp,
                                            C.c_int], C.c_int),
            ("orc_kad_maintenance_round", [vp, vp, u64, vp, vp, vp, C.c_int], u64),
            ("orc_kad_export_csr", [vp, vp, vp, vp], None),
            ("orc_kad_routing_add", [vp, u32, u32, C.c_int], C.c_int),
            ("orc_kad_build_tables_csr", [vp, u32, vp, vp, vp, vp, vp], vp),
            ("orc_kad_bucket_size", [vp, C.c_int], C.c_int),
            ("orc_kad_num_buckets", [vp], C.c_int),
            ("orc_epichord_find_node", [vp, u32, u32, vp, C.c_int, vp, C.c_int, C.c_int, C.c_int, vp, vp, vp,
                                        C.c_int, vp, u32, C.c_int64, C.c_int64, C.c_int, vp, vp, C.c_int], C.c_int),
            ("orc_kbrtest_lookup_stats", [vp, vp, vp, C.c_int, vp, vp, u64, C.c_double, C.c_int, C.c_double, vp],
             None),
        ]:
            f = getattr(L, name)
            f.argtypes = args
            f.restype = res
        _L = L
    return _L


class OrcKadRoundStats(C.Structure):
    _fields_ = [(f, C.c_uint64) for f in ("lookups", "failed", "responses", "sib_changes", "bucket_changes", "lost",
                                           "replacement", "refreshed")]


class OrcStdDev(C.Structure):
    _fields_ = [("count", C.c_uint64), ("mean", C.c_double), ("stddev", C.c_double),
                ("min", C.c_double), ("max", C.c_double)]


class OrcKbrTestResult(C.Structure):
    _fields_ = [("num_sent", C.c_uint64), ("num_delivered", C.c_uint64), ("num_dropped", C.c_uint64),
                ("num_lookup_failed", C.c_uint64), ("hop_count_sum", C.c_uint64), ("latency_sum_ns", C.c_int64),
                ("hop_count_mean", C.c_double), ("latency_mean_s", C.c_double), ("sd", OrcStdDev * 5)]


class OrcKbrTestLookupResult(C.Structure):
    _fields_ = [("num_sent", C.c_uint64), ("num_success", C.c_uint64), ("num_failed", C.c_uint64),
                ("num_invalid", C.c_uint64), ("hop_count_sum", C.c_uint64), ("failed_hop_count_sum", C.c_uint64),
                ("success_latency_sum_ns", C.c_int64), ("hop_count_mean", C.c_double),
                ("failed_hop_count_mean", C.c_double), ("success_latency_mean_s", C.c_double),
                ("total_latency_mean_s", C.c_double), ("sd", OrcStdDev * 3)]


LOOKUP_SD_FIELDS = ("successful_lookups_per_s", "failed_lookups_per_s", "success_ratio")

SD_FIELDS = ("delivered_msgs_per_s", "delivered_bytes_per_s", "dropped_msgs_per_s", "dropped_bytes_per_s",
             "delivery_ratio")


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def chord_params(**kw) -> OrcParams:
    p = OrcParams()
    lib().orc_params_chord_default(C.byref(p))
    return p.replace(**kw) if kw else p


def kad_params(**kw) -> OrcParams:
    p = OrcParams()
    lib().orc_params_kad_default(C.byref(p))
    return p.replace(**kw) if kw else p


def koorde_params(**kw) -> OrcParams:
    p = OrcParams()
    lib().orc_params_koorde_default(C.byref(p))
    return p.replace(**kw) if kw else p


class OracleNet:
    """A network built by the oracle (Chord stable state, Kademlia snapshot, converged Koorde)."""

    def __init__(self, kind: str, ids, xy, params: OrcParams | None = None, tables: dict | None = None,
                 lazy: bool = False):
        """lazy: store no tables, evaluate them per access (orc_*_build_lazy) -- same results, O(n)
        memory, for samples of the 2^26-node Chord (D) and 2^24-node Kademlia (E) networks."""
        self.ids = np.ascontiguousarray(ids, dtype=np.uint32)
        self.xy = np.ascontiguousarray(xy, dtype=np.float64)
        self.kind = kind
        L = lib()
        n = len(self.ids)
        if kind == "chord":
            self.params = params or chord_params()
            if tables is None:
                build = L.orc_chord_build_lazy if lazy else L.orc_chord_build
                h = build(_p(self.ids), n, _p(self.xy), C.byref(self.params))
            else:
                t = {k: np.ascontiguousarray(v) for k, v in tables.items()}
                self._keep = t
                h = L.orc_chord_build_tables(_p(self.ids), n, _p(self.xy), _p(t["pred"].astype(np.uint32)),
                                             _p(t["succ"]), _p(t["nsucc"]), t["succ"].shape[1], _p(t["fingers"]),
                                             _p(t["deque_size"]), C.byref(self.params))
        elif kind == "koorde":
            self.params = params or koorde_params()
            h = L.orc_koorde_build(_p(self.ids), n, _p(self.xy), C.byref(self.params))
        else:
            self.params = params or kad_params()
            if tables is None:
                build = L.orc_kad_build_lazy if lazy else L.orc_kad_build
                h = build(_p(self.ids), n, _p(self.xy), C.byref(self.params))
            elif "bucket_off" in tables:       # CSR tables: any b, any bucket size
                t = {k: np.ascontiguousarray(v) for k, v in tables.items()}
                t["siblings"] = t["siblings"].astype(np.uint32)
                t["bucket_off"] = t["bucket_off"].astype(np.uint64)
                t["bucket_nodes"] = np.ascontiguousarray(t["bucket_nodes"].astype(np.uint32))
                self._keep = t
                h = L.orc_kad_build_tables_csr(_p(self.ids), n, _p(self.xy), _p(t["siblings"]), _p(t["bucket_off"]),
                                               _p(t["bucket_nodes"]), C.byref(self.params))
            else:
                t = {k: np.ascontiguousarray(v) for k, v in tables.items()}
                self._keep = t
                h = L.orc_kad_build_tables(_p(self.ids), n, _p(self.xy), _p(t["siblings"].astype(np.uint32)),
                                           _p(t["bucket_count"].astype(np.uint8)),
                                           _p(t["bucket_nodes"].astype(np.uint32)), C.byref(self.params))
        if not h:
            raise RuntimeError(f"oracle build failed: {L.orc_last_error().decode()}")
        self._h = C.c_void_p(h)
        self.n = n

    def __del__(self):
        if getattr(self, "_h", None):
            lib().orc_net_free(self._h)
            self._h = None

    def route(self, keys, src, record_hops=True, count_rpcs=False, nthreads=0) -> dict:
        keys = np.ascontiguousarray(keys, dtype=np.uint32)
        src = np.ascontiguousarray(src, dtype=np.uint32)
        n = len(keys)
        out = np.empty(n, dtype=ROUTE_DTYPE)
        H = max(self.params.hopCountMax, 1)
        hop = np.empty((n, H), dtype=np.uint32) if record_hops else None
        rpcs = np.empty(n, dtype=np.uint32) if count_rpcs else None
        if lib().orc_route_batch(self._h, _p(keys), _p(src), n, _p(out), _p(hop), _p(rpcs), nthreads) == ORC_FAIL:
            raise RuntimeError(f"oracle: {lib().orc_last_error().decode()}")
        res = {f: out[f].copy() for f in ROUTE_DTYPE.names}
        if hop is not None:
            res["hop_seq"] = hop
        if rpcs is not None:
            res["rpcs"] = rpcs
        return res

    def lookup_call(self, keys, src, numSiblings: int = -1, nthreads=0) -> dict:
        """Batched LookupCalls (orc_lookup_batch); numSiblings = -1 is getMaxNumSiblings()."""
        keys = np.ascontiguousarray(keys, dtype=np.uint32)
        src = np.ascontiguousarray(src, dtype=np.uint32)
        n = len(keys)
        ns = numSiblings if numSiblings >= 0 else (self.params.s if self.kind == "kademlia"
                                                   else self.params.successorListSize)
        out = np.empty(n, dtype=LOOKUP_DTYPE)
        sib = np.empty((n, max(ns, 1)), dtype=np.uint32)
        r = lib().orc_lookup_batch(self._h, _p(keys), _p(src), n, numSiblings, _p(out), _p(sib), nthreads)
        if r < 0:
            raise ValueError(lib().orc_last_error().decode())
        res = {f: out[f].copy() for f in LOOKUP_DTYPE.names}
        res["siblings"] = sib
        return res

    def exhaustive(self, keys, src, R: int, record=True, nthreads=0) -> dict:
        """Exhaustive-iterative refresh lookups (orc_kad_exhaustive_batch) with redundantNodes = R."""
        keys = np.ascontiguousarray(keys, dtype=np.uint32)
        src = np.ascontiguousarray(src, dtype=np.uint32)
        n = len(keys)
        H = max(self.params.hopCountMax, 1)
        out = np.empty(n, dtype=LOOKUP_DTYPE)
        sib = np.empty((n, R), dtype=np.uint32)
        resp = np.empty((n, H), dtype=np.uint32) if record else None
        rtt = np.empty((n, H), dtype=np.int64) if record else None
        rpcs = np.empty(n, dtype=np.uint32)
        r = lib().orc_kad_exhaustive_batch(self._h, _p(keys), _p(src), n, R, _p(out), _p(sib), _p(resp), _p(rtt),
                                           _p(rpcs), nthreads)
        if r < 0:
            raise ValueError(lib().orc_last_error().decode())
        res = {f: out[f].copy() for f in LOOKUP_DTYPE.names}
        res["siblings"] = sib
        res["rpcs"] = rpcs
        if record:
            res["responders"] = resp
            res["rtt_ns"] = rtt
        return res

    def exhaustive_times(self, keys, src, R: int, ccap: int | None = None, nthreads=0) -> dict:
        """exhaustive() plus each accepted response's arrival at the source (tarr_ns) and every
        FindNodeCall sent (call_node, call_ns: its arrival at the destination), ns from the
        lookup's start (orc_kad_exhaustive_batch_t)."""
        keys = np.ascontiguousarray(keys, dtype=np.uint32)
        src = np.ascontiguousarray(src, dtype=np.uint32)
        n = len(keys)
        H = max(self.params.hopCountMax, 1)
        ccap = ccap or (2 * H + 2 * self.params.lookupParallelRpcs + 16)
        out = np.empty(n, dtype=LOOKUP_DTYPE)
        sib = np.empty((n, R), dtype=np.uint32)
        resp = np.empty((n, H), dtype=np.uint32)
        rtt, ta = (np.empty((n, H), dtype=np.int64) for _ in range(2))
        cn = np.empty((n, ccap), dtype=np.uint32)
        ct = np.empty((n, ccap), dtype=np.int64)
        rpcs = np.empty(n, dtype=np.uint32)
        r = lib().orc_kad_exhaustive_batch_t(self._h, _p(keys), _p(src), n, R, _p(out), _p(sib), _p(resp), _p(rtt),
                                             _p(ta), _p(cn), _p(ct), ccap, _p(rpcs), nthreads)
        if r < 0:
            raise ValueError(lib().orc_last_error().decode())
        res = {f: out[f].copy() for f in LOOKUP_DTYPE.names}
        res.update(siblings=sib, rpcs=rpcs, responders=resp, rtt_ns=rtt, tarr_ns=ta, call_node=cn, call_ns=ct)
        return res

    def maintenance_round(self, nodes=None, flags=None, stale=None, nthreads=0) -> dict:
        """One synchronous Kademlia maintenance round (orc_kad_maintenance_round) on explicit tables:
        the listed nodes' refresh lookups, then routingAdd at every node; returns its counters."""
        nodes = np.arange(self.n, dtype=np.uint32) if nodes is None else np.ascontiguousarray(nodes, np.uint32)
        fl = None if flags is None else np.ascontiguousarray(np.broadcast_to(flags, nodes.shape), dtype=np.uint8)
        st = None if stale is None else np.ascontiguousarray(stale, dtype=np.uint32)
        stats = OrcKadRoundStats()
        r = lib().orc_kad_maintenance_round(self._h, _p(nodes), len(nodes), _p(fl), _p(st), C.byref(stats), nthreads)
        if r == ORC_FAIL:
            raise RuntimeError(lib().orc_last_error().decode())
        d = {f: getattr(stats, f) for f, _ in OrcKadRoundStats._fields_}
        d["changes"] = int(r)
        return d

    def routing_add(self, v: int, x: int, alive: bool = True) -> int:
        r = lib().orc_kad_routing_add(self._h, int(v), int(x), int(bool(alive)))
        if r < 0:
            raise RuntimeError(lib().orc_last_error().decode())
        return r

    def num_buckets(self) -> int:
        return int(lib().orc_kad_num_buckets(C.byref(self.params)))

    def kad_tables_csr(self):
        """(siblings[n, 5s], bucket_off[n*NB+1], bucket_nodes) -- buckets of any size, LRU order;
        NB = numBuckets = (2^b - 1) * (160 / b)."""
        sib = np.empty((self.n, 5 * self.params.s), dtype=np.uint32)
        off = np.empty(self.n * self.num_buckets() + 1, dtype=np.uint64)
        lib().orc_kad_export_csr(self._h, _p(sib), _p(off), None)
        nodes = np.empty(max(int(off[-1]), 1), dtype=np.uint32)
        lib().orc_kad_export_csr(self._h, _p(sib), _p(off), _p(nodes))
        return sib, off, nodes[: int(off[-1])]

    def refresh_keys(self, nodes, stale=None):
        """Bucket-refresh (key, src) pairs of Kademlia::handleBucketRefreshTimerExpired."""
        nodes = np.ascontiguousarray(nodes, dtype=np.uint32)
        st = None if stale is None else np.ascontiguousarray(stale, dtype=np.uint32)
        L = lib()
        cnt = L.orc_kad_refresh_keys(self._h, _p(nodes), len(nodes), _p(st), None, None, 0)
        if cnt == ORC_FAIL:
            raise ValueError(L.orc_last_error().decode())
        keys = np.zeros((max(cnt, 1), 5), dtype=np.uint32)
        src = np.zeros(max(cnt, 1), dtype=np.uint32)
        L.orc_kad_refresh_keys(self._h, _p(nodes), len(nodes), _p(st), _p(keys), _p(src), cnt)
        return keys[:cnt], src[:cnt]

    def kbrtest_stats(self, result: dict, keys, src, measured_time_s: float, lookupNodeIds: bool = True,
                      testMsgSize: int = 100) -> dict:
        out = np.empty(len(result["responsible"]), dtype=ROUTE_DTYPE)
        for f in ROUTE_DTYPE.names:
            out[f] = result[f]
        keys = np.ascontiguousarray(keys, dtype=np.uint32)
        src = np.ascontiguousarray(src, dtype=np.uint32)
        st = OrcKbrTestResult()
        lib().orc_kbrtest_stats(self._h, _p(out), _p(keys), _p(src), len(out), float(measured_time_s),
                                int(bool(lookupNodeIds)), int(testMsgSize), C.byref(st))
        d = {f: getattr(st, f) for f, _ in OrcKbrTestResult._fields_ if f != "sd"}
        for i, name in enumerate(SD_FIELDS):
            s = st.sd[i]
            d[name] = {"count": s.count, "mean": s.mean, "stddev": s.stddev, "min": s.min, "max": s.max}
        return d

    def kbrtest_lookup_stats(self, result: dict, keys, src, measured_time_s: float, lookupNodeIds: bool = True,
                             failureLatency: float = 10.0) -> dict:
        out = np.empty(len(result["hops"]), dtype=LOOKUP_DTYPE)
        for f in LOOKUP_DTYPE.names:
            out[f] = result[f]
        sib = np.ascontiguousarray(result["siblings"], dtype=np.uint32)
        keys = np.ascontiguousarray(keys, dtype=np.uint32)
        src = np.ascontiguousarray(src, dtype=np.uint32)
        st = OrcKbrTestLookupResult()
        lib().orc_kbrtest_lookup_stats(self._h, _p(out), _p(sib), sib.shape[1], _p(keys), _p(src), len(out),
                                       float(measured_time_s), int(bool(lookupNodeIds)), float(failureLatency),
                                       C.byref(st))
        d = {f: getattr(st, f) for f, _ in OrcKbrTestLookupResult._fields_ if f != "sd"}
        for i, name in enumerate(LOOKUP_SD_FIELDS):
            s = st.sd[i]
            d[name] = {"count": s.count, "mean": s.mean, "stddev": s.stddev, "min": s.min, "max": s.max}
        return d

    def find_node(self, node: int, key, numRedundantNodes: int, numSiblings: int):
        key = np.ascontiguousarray(key, dtype=np.uint32)
        out = np.empty(64, dtype=np.uint32)
        flag = C.c_int(0)
        cnt = lib().orc_find_node(self._h, int(node), _p(key), numRedundantNodes, numSiblings, _p(out), C.byref(flag))
        return list(out[:cnt]), bool(flag.value)

    def chord_fix_fingers(self, nodes=None, nthreads=0) -> dict:
        """One synchronous fixfingers round (orc_chord_fix_fingers); returns its counters."""
        nodes = np.arange(self.n, dtype=np.uint32) if nodes is None else np.ascontiguousarray(nodes, np.uint32)
        ok, ch = C.c_uint64(0), C.c_uint64(0)
        hops = lib().orc_chord_fix_fingers(self._h, _p(nodes), len(nodes), C.byref(ok), C.byref(ch), nthreads)
        return {"hops": int(hops), "ok": ok.value, "changed": ch.value}

    def chord_stabilize(self, nodes=None) -> dict:
        """One synchronous stabilize round (orc_chord_stabilize) on explicit tables."""
        nodes = np.arange(self.n, dtype=np.uint32) if nodes is None else np.ascontiguousarray(nodes, np.uint32)
        sc, pc = C.c_uint64(0), C.c_uint64(0)
        r = lib().orc_chord_stabilize(self._h, _p(nodes), len(nodes), C.byref(sc), C.byref(pc))
        if r == ORC_FAIL:
            raise RuntimeError(lib().orc_last_error().decode())
        return {"nodes": len(nodes), "lists_changed": int(r), "succ_changed": sc.value, "pred_changed": pc.value}

    def chord_lists(self):
        sls = self.params.successorListSize
        pred = np.empty(self.n, dtype=np.uint32)
        succ = np.empty((self.n, sls), dtype=np.uint32)
        nsucc = np.empty(self.n, dtype=np.uint8)
        lib().orc_chord_export_lists(self._h, _p(pred), _p(succ), _p(nsucc))
        return pred, succ, nsucc

    def chord_fingers(self) -> np.ndarray:
        out = np.empty((self.n, 160), dtype=np.uint32)
        lib().orc_chord_export_fingers(self._h, _p(out))
        return out

    def kad_tables(self):
        sib = np.empty((self.n, 5 * self.params.s), dtype=np.uint32)
        cnt = np.empty((self.n, 160), dtype=np.uint8)
        nodes = np.empty((self.n, 160, self.params.k), dtype=np.uint32)
        lib().orc_kad_export(self._h, _p(sib), _p(cnt), _p(nodes))
        return sib, cnt, nodes

    def koorde_state(self):
        """(deBruijnNode, first node of the de Bruijn list, list length) per node."""
        db = np.empty(self.n, dtype=np.uint32)
        start = np.empty(self.n, dtype=np.uint32)
        num = np.empty(self.n, dtype=np.uint8)
        lib().orc_koorde_export(self._h, _p(db), _p(start), _p(num))
        return db, start, num

    def koorde_find_node(self, node: int, key, route_key=None, step: int = 1):
        """Koorde::findNode with a KoordeFindNodeExtMessage (route_key None = unspecified):
        returns (next hop or None when the reference throws, route_key out, step out)."""
        key = np.ascontiguousarray(key, dtype=np.uint32)
        rk = np.zeros(5, dtype=np.uint32) if route_key is None else np.array(route_key, dtype=np.uint32)
        has, st = C.c_int(0 if route_key is None else 1), C.c_int(step)
        h = lib().orc_koorde_find_node(self._h, int(node), _p(key), _p(rk), C.byref(has), C.byref(st))
        return (None if h == 0xFFFFFFFF else int(h)), (rk.copy() if has.value else None), st.value

    def delay_ns(self, a: int, b: int, nbytes: int) -> int:
        return int(lib().orc_delay_ns(self._h, a, b, nbytes))


def epichord_find_node(snap: dict, node: int, key, src: int, now: int, R: int, cap: int | None = None):
    """orc_epichord_find_node on a tests/epichord_snap.py snapshot: (status, nodes, lastUpdates);
    status = the count, -1 the reference throws, -2 it dereferences an empty cache."""
    L = lib()
    cap = cap or max(3, 1 + R)
    o0, o1 = int(snap["cache_off"][node]), int(snap["cache_off"][node + 1])
    cn = np.ascontiguousarray(snap["cache_node"][o0:o1])
    cl = np.ascontiguousarray(snap["cache_last"][o0:o1])
    ct = np.ascontiguousarray(snap["cache_ttl"][o0:o1])
    succ = np.ascontiguousarray(snap["succ"][node])
    pred = np.ascontiguousarray(snap["pred"][node])
    k = np.ascontiguousarray(np.asarray(key, dtype=np.uint32).reshape(5))
    out = np.full(cap, 0xFFFFFFFF, dtype=np.uint32)
    last = np.full(cap, -1, dtype=np.int64)
    ids = np.ascontiguousarray(snap["ids"], dtype=np.uint32)
    r = L.orc_epichord_find_node(_p(ids), snap["n"], int(node), _p(succ), int(snap["nsucc"][node]), _p(pred),
                                 int(snap["npred"][node]), int(snap["full"][node]), snap["L"], _p(cn), _p(cl), _p(ct),
                                 o1 - o0, _p(k), int(src), int(now), int(snap["cache_ttl_param"]), int(R), _p(out),
                                 _p(last), cap)
    if r == -3 or r == -4:
        raise ValueError(f"orc_epichord_find_node: bad input ({r})")
    m = max(r, 0)
    return r, out[:m].copy(), last[:m].copy()
