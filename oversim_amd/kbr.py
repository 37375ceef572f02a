"""Host-side mirror of OverSim's KBR lookup interface over the C ABI (include/ovs_kbr.h).

Names follow the reference so a test reads like OverSim code:

  KbrEngine.lookupCall(keys, src, numSiblings)
        -> BaseOverlay::lookupRpc for a batch of KBRTestApp LookupCalls
           (KBRTestApp.cc:190-206, BaseOverlay.cc:1938-1968, 1272-1300)
  KbrEngine.findNode(node, key, numRedundantNodes, numSiblings)
        -> BaseOverlay::findNode (BaseOverlay.h:693-696; Chord.cc:548-599,
           Kademlia.cc:1101-1246), evaluated at `node`
  KbrEngine.isSiblingFor(node, key, numSiblings)
        -> BaseOverlay::isSiblingFor (BaseOverlay.h:417-418), node == thisNode
  KbrEngine.lookup(keys, src)
        -> AbstractLookup::lookup + LookupListener::lookupFinished for a batch
           of KBRTestApp one-way tests (IterativeLookup.cc:695-723,
           BaseOverlay.cc:1241-1307)

Errors raised by the engine become KbrError (the reference throws
cRuntimeError).  There is no CPU fallback: importing this module without the
built HIP library raises.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass
from pathlib import Path

import numpy as np

# OVS_LIB selects an experimental build of the same engine (tools/build_alt_src.sh); default: the in-tree build
_LIB_PATH = Path(os.environ.get("OVS_LIB") or Path(__file__).resolve().parent / "libovs_kbr.so")

OVERLAY_CHORD = 1
OVERLAY_KADEMLIA = 2
OVERLAY_KOORDE = 3
OVERLAY_EPICHORD = 4
DEVICE_PTRS = 0x1
NONE = 0xFFFFFFFF

STATUS = {0: "OK", 1: "EINVAL", 2: "ENOMEM", 3: "EDEVICE", 4: "ESTATE", 5: "ENOTSUP"}
LOOKUP_STATUS = {0: "OK", 1: "TIMEOUT", 2: "RPC_TIMEOUT", 3: "HOPMAX", 4: "NO_NEXT", 5: "BROKEN", 6: "INVALID"}


class KbrError(RuntimeError):
    """cRuntimeError equivalent raised from an ovs_status != OVS_OK."""


class Params(C.Structure):
    """ovs_params; field names are the NED/.ini parameter names."""

    _fields_ = [
        ("overlay", C.c_int32), ("keyLength", C.c_int32), ("hopCountMax", C.c_int32),
        ("successorListSize", C.c_int32), ("extendedFingerTable", C.c_int32),
        ("numFingerCandidates", C.c_int32), ("k", C.c_int32), ("s", C.c_int32), ("b", C.c_int32),
        ("lookupRedundantNodes", C.c_int32), ("lookupParallelPaths", C.c_int32),
        ("lookupParallelRpcs", C.c_int32), ("lookupMerge", C.c_int32),
        ("lookupStrictParallelRpcs", C.c_int32), ("lookupVisitOnlyOnce", C.c_int32),
        ("lookupAcceptLateSiblings", C.c_int32), ("lookupUseAllParallelResponses", C.c_int32),
        ("lookupNewRpcOnEveryTimeout", C.c_int32), ("lookupNewRpcOnEveryResponse", C.c_int32),
        ("lookupFinishOnFirstUnchanged", C.c_int32), ("lookupVerifySiblings", C.c_int32),
        ("lookupMajoritySiblings", C.c_int32), ("routingType", C.c_int32), ("numSiblings", C.c_int32),
        ("useCoordinateBasedDelay", C.c_int32), ("simtimeRound", C.c_int32), ("testMsgSize", C.c_int32),
        ("recNumRedundantNodes", C.c_int32), ("rpcUdpTimeout", C.c_double), ("lookupTimeout", C.c_double),
        ("jitter", C.c_double), ("constantDelay", C.c_double), ("datarate", C.c_double),
        ("accessDelay", C.c_double), ("kadSeed", C.c_uint64),
        ("shiftingBits", C.c_int32), ("deBruijnListSize", C.c_int32), ("useOtherLookup", C.c_int32),
        ("useSucList", C.c_int32), ("bucketType", C.c_int32), ("cacheTTL", C.c_double),
        ("globalNodeLimit", C.c_int32), ("extraNodesFinalBucket", C.c_int32), ("rpcKeyTimeout", C.c_double),
        ("measureAuthBlock", C.c_int32),
    ]

    @classmethod
    def default(cls, overlay: int = OVERLAY_CHORD) -> "Params":
        p = cls()
        lib().ovs_params_default(overlay, C.byref(p))
        return p

    @classmethod
    def chord(cls) -> "Params":
        return cls.default(OVERLAY_CHORD)

    @classmethod
    def kademlia(cls) -> "Params":
        return cls.default(OVERLAY_KADEMLIA)

    @classmethod
    def koorde(cls) -> "Params":
        return cls.default(OVERLAY_KOORDE)

    @classmethod
    def epichord(cls) -> "Params":
        return cls.default(OVERLAY_EPICHORD)

    @classmethod
    def from_ini(cls, text: str, config: str | None = None, overlay: int = OVERLAY_CHORD,
                 base: "Params | None" = None) -> "Params":
        p = cls()
        C.memmove(C.byref(p), C.byref(base), C.sizeof(cls)) if base is not None else lib().ovs_params_default(overlay, C.byref(p))
        err = C.create_string_buffer(512)
        st = lib().ovs_params_from_ini(C.byref(p), text.encode(), config.encode() if config else None, err, 512)
        if st != 0:
            raise KbrError(f"ovs_params_from_ini: {STATUS.get(st, st)}: {err.value.decode()}")
        return p

    @classmethod
    def from_ini_file(cls, path, config: str | None = None, overlay: int = OVERLAY_CHORD) -> "Params":
        """Like from_ini, reading the file and its `include` lines as Cmdenv does."""
        p = cls()
        lib().ovs_params_default(overlay, C.byref(p))
        err = C.create_string_buffer(512)
        st = lib().ovs_params_from_ini_file(C.byref(p), str(path).encode(), config.encode() if config else None, err, 512)
        if st != 0:
            raise KbrError(f"ovs_params_from_ini_file: {STATUS.get(st, st)}: {err.value.decode()}")
        return p

    def as_dict(self) -> dict:
        return {f: getattr(self, f) for f, _ in self._fields_ if not f.startswith("_")}

    def replace(self, **kw) -> "Params":
        p = Params()
        C.memmove(C.byref(p), C.byref(self), C.sizeof(Params))
        for k, v in kw.items():
            setattr(p, k, v)
        return p


ROUTE_OUT_DTYPE = np.dtype([("responsible", "<u4"), ("hops", "<u2"), ("status", "u1"),
                            ("one_way_hops", "u1"), ("latency_ns", "<i8")])
assert ROUTE_OUT_DTYPE.itemsize == 16
KOORDE_EXT_DTYPE = np.dtype([("route_key", "<u4", 5), ("step", "<i4"), ("has_route_key", "<i4")])
assert KOORDE_EXT_DTYPE.itemsize == 28
LOOKUP_OUT_DTYPE = np.dtype([("num_siblings", "<u4"), ("hops", "<u2"), ("status", "u1"),
                             ("is_valid", "u1"), ("latency_ns", "<i8")])
assert LOOKUP_OUT_DTYPE.itemsize == 16

class StdDev(C.Structure):
    """ovs_stddev: one cStdDev summary (GlobalStatistics::addStdDev)."""

    _fields_ = [("count", C.c_uint64), ("mean", C.c_double), ("stddev", C.c_double),
                ("min", C.c_double), ("max", C.c_double)]


class KbrTestStats(C.Structure):
    """ovs_kbrtest_stats: KBRTestApp one-way statistics of a batch (KBRTestApp.cc:380-520)."""

    _fields_ = [
        ("num_sent", C.c_uint64), ("num_delivered", C.c_uint64), ("num_dropped", C.c_uint64),
        ("num_lookup_failed", C.c_uint64), ("bytes_sent", C.c_uint64), ("bytes_delivered", C.c_uint64),
        ("bytes_dropped", C.c_uint64), ("hop_count_sum", C.c_uint64), ("latency_sum_ns", C.c_int64),
        ("hop_count_min", C.c_uint32), ("hop_count_max", C.c_uint32),
        ("latency_min_ns", C.c_int64), ("latency_max_ns", C.c_int64),
        ("hop_count_mean", C.c_double), ("latency_mean_s", C.c_double),
        ("status_count", C.c_uint64 * 8), ("hop_hist", C.c_uint64 * 64),
        ("delivered_msgs_per_s", StdDev), ("delivered_bytes_per_s", StdDev),
        ("dropped_msgs_per_s", StdDev), ("dropped_bytes_per_s", StdDev), ("delivery_ratio", StdDev),
    ]

    STDDEV_NAMES = {
        "delivered_msgs_per_s": "KBRTestApp: One-way Delivered Messages/s",
        "delivered_bytes_per_s": "KBRTestApp: One-way Delivered Bytes/s",
        "dropped_msgs_per_s": "KBRTestApp: One-way Dropped Messages/s",
        "dropped_bytes_per_s": "KBRTestApp: One-way Dropped Bytes/s",
        "delivery_ratio": "KBRTestApp: One-way Delivery Ratio",
    }


_lib = None


def lib() -> C.CDLL:
    """Load libovs_kbr.so; raises if the HIP engine was not built (no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not _LIB_PATH.exists():
        raise ImportError(f"{_LIB_PATH} missing: run `python -c 'import __graft_entry__ as g; g.build()'` "
                          "(the MI355X engine has no CPU fallback)")
    # One HIP runtime per process: PyTorch ships its own libamdhip64 / libhsa-runtime64 (same
    # SONAMEs as /opt/rocm's).  Loaded after torch, the engine binds to torch's copies; loaded
    # before it, torch would map a second runtime and whichever initialises second finds no GPU
    # (tools/diag/runtime_order.py).  So torch, when installed, is imported first.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(str(_LIB_PATH))
    L.ovs_build_id.argtypes = []
    L.ovs_build_id.restype = C.c_char_p
    if not os.environ.get("OVS_LIB"):
        # the library must be the build of the sources it ships with (oversim_amd/build.py)
        from .build import source_hash
        built, want = L.ovs_build_id().decode(), source_hash()
        if built != want:
            raise ImportError(f"{_LIB_PATH} is stale (build id {built}, sources {want}): rebuild with "
                              "`python -m oversim_amd.build`")
    vp, u64, u32, i32 = C.c_void_p, C.c_uint64, C.c_uint32, C.c_int32
    sigs = {
        "ovs_abi_version": ([], C.c_int),
        "ovs_params_default": ([i32, vp], None),
        "ovs_params_from_ini": ([vp, C.c_char_p, C.c_char_p, C.c_char_p, C.c_int], C.c_int),
        "ovs_params_from_ini_file": ([vp, C.c_char_p, C.c_char_p, C.c_char_p, C.c_int], C.c_int),
        "ovs_ctx_create": ([C.c_int, C.POINTER(vp)], C.c_int),
        "ovs_ctx_destroy": ([vp], None),
        "ovs_last_error": ([vp], C.c_char_p),
        "ovs_set_params": ([vp, vp], C.c_int),
        "ovs_get_params": ([vp, vp], C.c_int),
        "ovs_chord_load": ([vp, vp, u64, vp, u32], C.c_int),
        "ovs_chord_load_tables": ([vp, vp, u64, vp, vp, vp, vp, vp, vp, u32], C.c_int),
        "ovs_kad_load": ([vp, vp, u64, vp, u32], C.c_int),
        "ovs_koorde_load": ([vp, vp, u64, vp, u32], C.c_int),
        "ovs_koorde_export": ([vp, vp, vp, vp], C.c_int),
        "ovs_koorde_find_node_batch": ([vp, vp, vp, vp, vp, u64], C.c_int),
        "ovs_kad_load_tables": ([vp, vp, u64, vp, vp, vp, vp, u32], C.c_int),
        "ovs_kad_num_buckets": ([vp], i32),
        "ovs_kad_load_tables_csr": ([vp, vp, u64, vp, vp, vp, vp, u32], C.c_int),
        "ovs_kad_export_csr": ([vp, vp, vp, vp, u64, C.POINTER(u64)], C.c_int),
        "ovs_epichord_load": ([vp, vp, u64, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, u32], C.c_int),
        "ovs_epichord_find_node_batch": ([vp, vp, vp, vp, vp, u64, i32, vp, vp, u32, vp, vp, u32, vp], C.c_int),
        "ovs_kad_export": ([vp, vp, vp, vp], C.c_int),
        "ovs_chord_export_fingers": ([vp, vp], C.c_int),
        "ovs_route_batch": ([vp, vp, vp, u64, vp, vp, vp, u32, vp], C.c_int),
        "ovs_find_node_batch": ([vp, vp, vp, u64, i32, i32, vp, u32, vp, vp, u32, vp], C.c_int),
        "ovs_delay_batch": ([vp, vp, vp, vp, u64, vp, u32, vp], C.c_int),
        "ovs_sync": ([vp], C.c_int),
        "ovs_kbrtest_stats_batch": ([vp, vp, vp, vp, u64, C.c_double, i32, vp, u32, vp], C.c_int),
        "ovs_chord_fix_fingers": ([vp, vp, u64, vp], C.c_int),
        "ovs_lookup_batch": ([vp, vp, vp, u64, i32, vp, vp, u32, vp], C.c_int),
        "ovs_chord_stabilize": ([vp, vp, u64, vp], C.c_int),
        "ovs_chord_export_tables": ([vp, vp, vp, vp], C.c_int),
        "ovs_kad_refresh_batch": ([vp, vp, vp, u64, i32, vp, vp, vp, vp, vp, u32, vp], C.c_int),
        "ovs_kad_refresh_keys": ([vp, vp, u64, vp, vp, vp, u64, C.POINTER(u64), u32, vp], C.c_int),
        "ovs_kad_maintenance_round": ([vp, vp, u64, vp, vp, vp], C.c_int),
        "ovs_kbrtest_lookup_stats_batch": ([vp, vp, vp, i32, vp, vp, u64, C.c_double, i32, C.c_double, vp, u32, vp],
                                           C.c_int),
    }
    for name, (args, res) in sigs.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    _lib = L
    return L


def _ptr(a: np.ndarray | None):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def keys_array(keys) -> np.ndarray:
    """(n,5) uint32 little-endian 32-bit words, w[0] least significant."""
    a = np.ascontiguousarray(keys, dtype=np.uint32)
    if a.ndim != 2 or a.shape[1] != 5:
        raise ValueError("keys must have shape (n, 5) uint32")
    return a


def key_from_int(x: int) -> np.ndarray:
    x &= (1 << 160) - 1
    return np.array([(x >> (32 * i)) & 0xFFFFFFFF for i in range(5)], dtype=np.uint32)


def key_to_int(w) -> int:
    return sum(int(w[i]) << (32 * i) for i in range(5))


class FixFingersStats(C.Structure):
    """ovs_fixfingers_stats: one fixfingers round (ovs_chord_fix_fingers)."""

    _fields_ = [("lookups", C.c_uint64), ("ok", C.c_uint64), ("changed", C.c_uint64), ("hops", C.c_uint64)]


class StabilizeStats(C.Structure):
    """ovs_stabilize_stats: one stabilize round (ovs_chord_stabilize)."""

    _fields_ = [("nodes", C.c_uint64), ("succ_changed", C.c_uint64), ("lists_changed", C.c_uint64),
                ("pred_changed", C.c_uint64)]


class KadRoundStats(C.Structure):
    """ovs_kad_round_stats: one Kademlia maintenance round (ovs_kad_maintenance_round)."""

    _fields_ = [(f, C.c_uint64) for f in ("lookups", "failed", "responses", "sib_changes", "bucket_changes", "lost",
                                           "replacement", "refreshed")]


class KbrTestLookupStats(C.Structure):
    """ovs_kbrtest_lookup_stats: KBRTestApp lookup-test statistics of a batch (KBRTestApp.cc:331-371, 546-557)."""

    _fields_ = [
        ("num_sent", C.c_uint64), ("num_success", C.c_uint64), ("num_failed", C.c_uint64),
        ("num_invalid", C.c_uint64), ("hop_count_sum", C.c_uint64), ("failed_hop_count_sum", C.c_uint64),
        ("success_latency_sum_ns", C.c_int64), ("hop_count_min", C.c_uint32), ("hop_count_max", C.c_uint32),
        ("success_latency_min_ns", C.c_int64), ("success_latency_max_ns", C.c_int64),
        ("hop_count_mean", C.c_double), ("failed_hop_count_mean", C.c_double),
        ("success_latency_mean_s", C.c_double), ("total_latency_mean_s", C.c_double),
        ("status_count", C.c_uint64 * 8), ("hop_hist", C.c_uint64 * 64),
        ("successful_lookups_per_s", StdDev), ("failed_lookups_per_s", StdDev), ("success_ratio", StdDev),
    ]

    STDDEV_NAMES = {
        "successful_lookups_per_s": "KBRTestApp: Successful Lookups/s",
        "failed_lookups_per_s": "KBRTestApp: Failed Lookups/s",
        "success_ratio": "KBRTestApp: Lookup Success Ratio",
    }


class KbrEngine:
    """One engine context per HIP device (ovs_ctx)."""

    def __init__(self, device: int = 0, params: Params | None = None):
        self._L = lib()
        h = C.c_void_p()
        st = self._L.ovs_ctx_create(device, C.byref(h))
        if st != 0:
            raise KbrError(f"ovs_ctx_create(device={device}) failed: {STATUS.get(st, st)}")
        self._h = h
        self.n = 0
        self.overlay = 0
        if params is not None:
            self.set_params(params)

    # -- plumbing
    def _chk(self, st: int, what: str):
        if st != 0:
            msg = self._L.ovs_last_error(self._h)
            raise KbrError(f"{what}: {STATUS.get(st, st)}: {msg.decode() if msg else ''}")

    def close(self):
        if getattr(self, "_h", None):
            self._L.ovs_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @property
    def handle(self) -> int:
        return self._h.value

    # -- parameters
    def set_params(self, p: Params):
        self._chk(self._L.ovs_set_params(self._h, C.byref(p)), "ovs_set_params")

    def get_params(self) -> Params:
        p = Params()
        self._chk(self._L.ovs_get_params(self._h, C.byref(p)), "ovs_get_params")
        return p

    # -- networks
    def chord_load(self, ids, xy):
        ids = keys_array(ids)
        xy = np.ascontiguousarray(xy, dtype=np.float64)
        self._chk(self._L.ovs_chord_load(self._h, _ptr(ids), len(ids), _ptr(xy), 0), "ovs_chord_load")
        self.n, self.overlay = len(ids), OVERLAY_CHORD

    def chord_load_device(self, ids_ptr: int, xy_ptr: int, n: int):
        """Load a Chord ring whose sorted ids / coordinates already live on this device."""
        self._chk(self._L.ovs_chord_load(self._h, C.c_void_p(ids_ptr), n, C.c_void_p(xy_ptr), DEVICE_PTRS),
                  "ovs_chord_load")
        self.n, self.overlay = n, OVERLAY_CHORD

    def koorde_load(self, ids, xy):
        """Converged Koorde ring (ovs_koorde_load); params.overlay must be OVERLAY_KOORDE."""
        ids = keys_array(ids)
        xy = np.ascontiguousarray(xy, dtype=np.float64)
        self._chk(self._L.ovs_koorde_load(self._h, _ptr(ids), len(ids), _ptr(xy), 0), "ovs_koorde_load")
        self.n, self.overlay = len(ids), OVERLAY_KOORDE

    def koorde_load_device(self, ids_ptr: int, xy_ptr: int, n: int):
        self._chk(self._L.ovs_koorde_load(self._h, C.c_void_p(ids_ptr), n, C.c_void_p(xy_ptr), DEVICE_PTRS),
                  "ovs_koorde_load")
        self.n, self.overlay = n, OVERLAY_KOORDE

    def koorde_state(self):
        """(deBruijnNode, first node of the deBruijnNodes list, list length) per node."""
        db = np.empty(self.n, dtype=np.uint32)
        start = np.empty(self.n, dtype=np.uint32)
        num = np.empty(self.n, dtype=np.uint8)
        self._chk(self._L.ovs_koorde_export(self._h, _ptr(db), _ptr(start), _ptr(num)), "ovs_koorde_export")
        return db, start, num

    def koorde_find_node(self, node, keys, ext=None):
        """Koorde::findNode at node[i] for keys[i]; ext = KOORDE_EXT_DTYPE records (None: fresh,
        unspecified route key, step 1) are advanced in place.  Returns (next hop, NONE where the
        reference throws; the extensions the responses carry)."""
        node = np.ascontiguousarray(node, dtype=np.uint32)
        keys = keys_array(keys)
        n = len(node)
        if ext is None:
            ext = np.zeros(n, dtype=KOORDE_EXT_DTYPE)
            ext["step"] = 1
        ext = np.ascontiguousarray(ext, dtype=KOORDE_EXT_DTYPE).copy()
        nxt = np.empty(n, dtype=np.uint32)
        self._chk(self._L.ovs_koorde_find_node_batch(self._h, _ptr(node), _ptr(keys), _ptr(ext), _ptr(nxt), n),
                  "ovs_koorde_find_node_batch")
        return nxt, ext

    def epichord_load(self, ids, xy, succ, nsucc, pred, npred, lists_full, cache_off, cache_node, cache_last_ns,
                      cache_ttl_ns):
        """One EpiChord routing snapshot (ovs_epichord_load): successor / predecessor lists (n, L) closest
        first with their lengths and isFull() bits, the live finger caches as CSR rows (node, lastUpdate,
        ttl in ns).  params.overlay must be OVERLAY_EPICHORD."""
        ids = keys_array(ids)
        arrs = [np.ascontiguousarray(a, dtype=t) for a, t in
                ((xy, np.float64), (succ, np.uint32), (nsucc, np.uint8), (pred, np.uint32), (npred, np.uint8),
                 (lists_full, np.uint8), (cache_off, np.uint64), (cache_node, np.uint32),
                 (cache_last_ns, np.int64), (cache_ttl_ns, np.int64))]
        self._chk(self._L.ovs_epichord_load(self._h, _ptr(ids), len(ids), *[_ptr(a) for a in arrs], 0),
                  "ovs_epichord_load")
        self.n, self.overlay = len(ids), OVERLAY_EPICHORD

    def epichord_find_node(self, node, keys, src, now_ns, numRedundantNodes: int, max_out: int | None = None):
        """EpiChord::findNode per call (ovs_epichord_find_node_batch): src NONE = a local call.  Returns
        (nodes (n, max_out), lastUpdates (n, max_out), count, status)."""
        node = np.ascontiguousarray(node, dtype=np.uint32)
        keys = keys_array(keys)
        src = np.ascontiguousarray(src, dtype=np.uint32)
        now = np.ascontiguousarray(now_ns, dtype=np.int64)
        n = len(node)
        mo = max_out or max(3, 1 + numRedundantNodes)
        out = np.empty((n, mo), dtype=np.uint32)
        last = np.empty((n, mo), dtype=np.int64)
        cnt = np.empty(n, dtype=np.uint8)
        st = np.empty(n, dtype=np.uint8)
        self._chk(self._L.ovs_epichord_find_node_batch(self._h, _ptr(node), _ptr(keys), _ptr(src), _ptr(now), n,
                                                       numRedundantNodes, _ptr(out), _ptr(last), mo, _ptr(cnt),
                                                       _ptr(st), 0, None), "ovs_epichord_find_node_batch")
        return out, last, cnt, st

    def kad_load_device(self, ids_ptr: int, xy_ptr: int, n: int):
        self._chk(self._L.ovs_kad_load(self._h, C.c_void_p(ids_ptr), n, C.c_void_p(xy_ptr), DEVICE_PTRS),
                  "ovs_kad_load")
        self.n, self.overlay = n, OVERLAY_KADEMLIA

    def chord_load_tables(self, ids, xy, pred, succ, nsucc, fingers, deque_size):
        ids = keys_array(ids)
        arrs = [np.ascontiguousarray(a, dtype=t) for a, t in
                ((xy, np.float64), (pred, np.uint32), (succ, np.uint32), (nsucc, np.uint8),
                 (fingers, np.uint32), (deque_size, np.uint8))]
        self._chk(self._L.ovs_chord_load_tables(self._h, _ptr(ids), len(ids), *[_ptr(a) for a in arrs], 0),
                  "ovs_chord_load_tables")
        self.n, self.overlay = len(ids), OVERLAY_CHORD

    def kad_load(self, ids, xy):
        ids = keys_array(ids)
        xy = np.ascontiguousarray(xy, dtype=np.float64)
        self._chk(self._L.ovs_kad_load(self._h, _ptr(ids), len(ids), _ptr(xy), 0), "ovs_kad_load")
        self.n, self.overlay = len(ids), OVERLAY_KADEMLIA

    def kad_load_tables(self, ids, xy, siblings, bucket_count, bucket_nodes):
        """Explicit Kademlia tables (ovs_kad_load_tables): siblings (n, 5s), bucket_count (n, 160),
        bucket_nodes (n, 160, k), 0xFFFFFFFF padded -- the k-buckets a running OverSim node holds."""
        ids = keys_array(ids)
        arrs = [np.ascontiguousarray(a, dtype=t) for a, t in
                ((xy, np.float64), (siblings, np.uint32), (bucket_count, np.uint8), (bucket_nodes, np.uint32))]
        self._chk(self._L.ovs_kad_load_tables(self._h, _ptr(ids), len(ids), *[_ptr(a) for a in arrs], 0),
                  "ovs_kad_load_tables")
        self.n, self.overlay = len(ids), OVERLAY_KADEMLIA

    def kad_load_tables_csr(self, ids, xy, siblings, bucket_off, bucket_nodes):
        """Kademlia tables in CSR form (ovs_kad_load_tables_csr): any b / bucketType of the current
        params -- siblings (n, 5s), bucket_off (n * numBuckets + 1) uint64, bucket_nodes (LRU order)."""
        ids = keys_array(ids)
        arrs = [np.ascontiguousarray(a, dtype=t) for a, t in
                ((xy, np.float64), (siblings, np.uint32), (bucket_off, np.uint64), (bucket_nodes, np.uint32))]
        self._chk(self._L.ovs_kad_load_tables_csr(self._h, _ptr(ids), len(ids), *[_ptr(a) for a in arrs], 0),
                  "ovs_kad_load_tables_csr")
        self.n, self.overlay = len(ids), OVERLAY_KADEMLIA

    def kad_num_buckets(self) -> int:
        p = self.get_params()
        return int(self._L.ovs_kad_num_buckets(C.byref(p)))

    def kad_tables_csr(self):
        """(siblings (n, 5s), bucket_off (n * numBuckets + 1), bucket_nodes) of the loaded tables."""
        p = self.get_params()
        nb = self.kad_num_buckets()
        sib = np.empty((self.n, 5 * p.s), dtype=np.uint32)
        off = np.empty(self.n * nb + 1, dtype=np.uint64)
        tot = C.c_uint64(0)
        self._chk(self._L.ovs_kad_export_csr(self._h, _ptr(sib), _ptr(off), None, 0, C.byref(tot)), "ovs_kad_export_csr")
        nodes = np.empty(max(int(tot.value), 1), dtype=np.uint32)
        self._chk(self._L.ovs_kad_export_csr(self._h, _ptr(sib), _ptr(off), _ptr(nodes), len(nodes), C.byref(tot)),
                  "ovs_kad_export_csr")
        return sib, off, nodes[:int(tot.value)]

    def chord_fingers(self) -> np.ndarray:
        out = np.empty((self.n, 160), dtype=np.uint32)
        self._chk(self._L.ovs_chord_export_fingers(self._h, _ptr(out)), "ovs_chord_export_fingers")
        return out

    def chord_fix_fingers(self, nodes=None) -> dict:
        """One synchronous fixfingers round on an explicit-table ring (ovs_chord_fix_fingers):
        the batched maintenance lookups of Chord::handleFixFingersTimerExpired."""
        nodes = np.arange(self.n, dtype=np.uint32) if nodes is None else np.ascontiguousarray(nodes, np.uint32)
        st = FixFingersStats()
        self._chk(self._L.ovs_chord_fix_fingers(self._h, _ptr(nodes), len(nodes), C.cast(C.byref(st), C.c_void_p)),
                  "ovs_chord_fix_fingers")
        return {f: getattr(st, f) for f, _ in FixFingersStats._fields_}

    def chord_stabilize(self, nodes=None) -> dict:
        """One synchronous stabilize round on an explicit-table ring (ovs_chord_stabilize): successor's
        predecessor, notify, successor-list update (Chord.cc:793-842, 1055-1225)."""
        nodes = np.arange(self.n, dtype=np.uint32) if nodes is None else np.ascontiguousarray(nodes, np.uint32)
        st = StabilizeStats()
        self._chk(self._L.ovs_chord_stabilize(self._h, _ptr(nodes), len(nodes), C.cast(C.byref(st), C.c_void_p)),
                  "ovs_chord_stabilize")
        return {f: getattr(st, f) for f, _ in StabilizeStats._fields_}

    def kad_maintenance_round(self, nodes=None, flags=None, stale=None) -> dict:
        """One synchronous Kademlia maintenance round (ovs_kad_maintenance_round): the listed nodes'
        refresh lookups on the device (flags bit 0 sibling refresh, bit 1 bucket refreshes; None =
        both), then Kademlia::routingAdd for every call and response on the host; returns the counters
        plus "changes" (membership changes)."""
        nodes = np.arange(self.n, dtype=np.uint32) if nodes is None else np.ascontiguousarray(nodes, np.uint32)
        fl = None if flags is None else np.ascontiguousarray(np.broadcast_to(flags, nodes.shape), dtype=np.uint8)
        stl = None if stale is None else np.ascontiguousarray(stale, dtype=np.uint32)
        st = KadRoundStats()
        self._chk(self._L.ovs_kad_maintenance_round(self._h, _ptr(nodes), len(nodes), _ptr(fl), _ptr(stl),
                                                    C.cast(C.byref(st), C.c_void_p)), "ovs_kad_maintenance_round")
        d = {f: getattr(st, f) for f, _ in KadRoundStats._fields_}
        d["changes"] = d["sib_changes"] + d["bucket_changes"] + d["lost"]
        return d

    def chord_tables(self):
        """(pred, succ (n, successorListSize), nsucc) of an explicit-table ring as they now stand."""
        sls = self.get_params().successorListSize
        pred = np.empty(self.n, dtype=np.uint32)
        succ = np.empty((self.n, sls), dtype=np.uint32)
        nsucc = np.empty(self.n, dtype=np.uint8)
        self._chk(self._L.ovs_chord_export_tables(self._h, _ptr(pred), _ptr(succ), _ptr(nsucc)),
                  "ovs_chord_export_tables")
        return pred, succ, nsucc

    def kad_tables(self):
        p = self.get_params()
        sib = np.empty((self.n, 5 * p.s), dtype=np.uint32)
        cnt = np.empty((self.n, 160), dtype=np.uint8)
        nodes = np.empty((self.n, 160, p.k), dtype=np.uint32)
        self._chk(self._L.ovs_kad_export(self._h, _ptr(sib), _ptr(cnt), _ptr(nodes)), "ovs_kad_export")
        return sib, cnt, nodes

    # -- the hot path
    def lookup(self, keys, src, record_hops: bool = False, count_rpcs: bool = False) -> dict:
        """Batched KBRTestApp one-way lookups; returns numpy arrays by field."""
        keys = keys_array(keys)
        src = np.ascontiguousarray(src, dtype=np.uint32)
        n = len(keys)
        if len(src) != n:
            raise ValueError("keys and src differ in length")
        out = np.empty(n, dtype=ROUTE_OUT_DTYPE)
        H = max(self.get_params().hopCountMax, 1)
        hop = np.empty((n, H), dtype=np.uint32) if record_hops else None
        rpcs = np.empty(n, dtype=np.uint32) if count_rpcs else None
        self._chk(self._L.ovs_route_batch(self._h, _ptr(keys), _ptr(src), n, _ptr(out), _ptr(hop), _ptr(rpcs), 0,
                                          None), "ovs_route_batch")
        res = {f: out[f].copy() for f in ROUTE_OUT_DTYPE.names}
        if hop is not None:
            res["hop_seq"] = hop
        if rpcs is not None:
            res["rpcs"] = rpcs
        return res

    def lookupCall(self, keys, src, numSiblings: int = -1) -> dict:
        """Batched LookupCalls (KBRTestApp lookup test; BaseOverlay::lookupRpc, BaseOverlay.cc:1938-1968,
        answered by SendToKeyListener::lookupFinished, 1272-1300).  numSiblings = -1 is
        getMaxNumSiblings(), as KBRTestApp sends it.  Returns num_siblings, hops, status, is_valid,
        latency_ns per lookup and `siblings` (n, numSiblings), NONE padded."""
        keys = keys_array(keys)
        src = np.ascontiguousarray(src, dtype=np.uint32)
        n = len(keys)
        if len(src) != n:
            raise ValueError("keys and src differ in length")
        p = self.get_params()
        ns = numSiblings if numSiblings >= 0 else (p.successorListSize if p.overlay == OVERLAY_CHORD else p.s)
        out = np.empty(n, dtype=LOOKUP_OUT_DTYPE)
        sib = np.empty((n, max(ns, 1)), dtype=np.uint32)
        self._chk(self._L.ovs_lookup_batch(self._h, _ptr(keys), _ptr(src), n, numSiblings, _ptr(out), _ptr(sib), 0,
                                           None), "ovs_lookup_batch")
        res = {f: out[f].copy() for f in LOOKUP_OUT_DTYPE.names}
        res["siblings"] = sib
        return res

    def kad_refresh(self, keys, src, redundantNodes: int, record: bool = True) -> dict:
        """Kademlia refresh lookups (ovs_kad_refresh_batch): exhaustive-iterative lookups of keys[i] from
        src[i] with config.redundantNodes = numSiblings = redundantNodes (Kademlia.cc:1591-1686).
        Returns the LookupCall fields, `siblings` (n, R), `rpcs`, and with record the responders
        (n, hopCountMax) and their RTTs in ns, in the order the responses arrived."""
        keys = keys_array(keys)
        src = np.ascontiguousarray(src, dtype=np.uint32)
        n = len(keys)
        if len(src) != n:
            raise ValueError("keys and src differ in length")
        R = int(redundantNodes)
        H = max(self.get_params().hopCountMax, 1)
        out = np.empty(n, dtype=LOOKUP_OUT_DTYPE)
        sib = np.empty((n, max(R, 1)), dtype=np.uint32)
        resp = np.empty((n, H), dtype=np.uint32) if record else None
        rtt = np.empty((n, H), dtype=np.int64) if record else None
        rpcs = np.empty(n, dtype=np.uint32)
        self._chk(self._L.ovs_kad_refresh_batch(self._h, _ptr(keys), _ptr(src), n, R, _ptr(out), _ptr(sib), _ptr(resp),
                                                _ptr(rtt), _ptr(rpcs), 0, None), "ovs_kad_refresh_batch")
        res = {f: out[f].copy() for f in LOOKUP_OUT_DTYPE.names}
        res["siblings"] = sib
        res["rpcs"] = rpcs
        if record:
            res["responders"] = resp
            res["rtt_ns"] = rtt
        return res

    def kad_refresh_device(self, keys_ptr: int, src_ptr: int, n: int, redundantNodes: int, out_ptr: int,
                           sib_ptr: int, rpcs_ptr: int | None = None, stream: int | None = None):
        """Device-resident refresh batch (no responder record)."""
        self._chk(self._L.ovs_kad_refresh_batch(self._h, C.c_void_p(keys_ptr), C.c_void_p(src_ptr), n, redundantNodes,
                                                C.c_void_p(out_ptr), C.c_void_p(sib_ptr), None, None,
                                                C.c_void_p(rpcs_ptr) if rpcs_ptr else None, DEVICE_PTRS,
                                                C.c_void_p(stream) if stream else None), "ovs_kad_refresh_batch")

    def kad_refresh_keys(self, nodes=None, stale=None):
        """The bucket-refresh (keys, src) of Kademlia::handleBucketRefreshTimerExpired for `nodes`
        (default: all); stale = (m, 5) uint32 bit masks of the buckets due (None: all)."""
        nodes = np.arange(self.n, dtype=np.uint32) if nodes is None else np.ascontiguousarray(nodes, np.uint32)
        st = None if stale is None else np.ascontiguousarray(stale, dtype=np.uint32)
        cnt = C.c_uint64(0)
        self._chk(self._L.ovs_kad_refresh_keys(self._h, _ptr(nodes), len(nodes), _ptr(st), None, None, 0,
                                               C.byref(cnt), 0, None), "ovs_kad_refresh_keys")
        total = cnt.value
        keys = np.zeros((max(total, 1), 5), dtype=np.uint32)
        src = np.zeros(max(total, 1), dtype=np.uint32)
        self._chk(self._L.ovs_kad_refresh_keys(self._h, _ptr(nodes), len(nodes), _ptr(st), _ptr(keys), _ptr(src),
                                               total, C.byref(cnt), 0, None), "ovs_kad_refresh_keys")
        return keys[:total], src[:total]

    def lookup_device(self, keys_ptr: int, src_ptr: int, n: int, out_ptr: int, stream: int | None = None,
                      hop_ptr: int | None = None, rpcs_ptr: int | None = None):
        """Device-resident batch (pointers on this context's device, async on `stream`, 0 = default stream)."""
        self._chk(self._L.ovs_route_batch(self._h, C.c_void_p(keys_ptr), C.c_void_p(src_ptr), n,
                                          C.c_void_p(out_ptr), C.c_void_p(hop_ptr) if hop_ptr else None,
                                          C.c_void_p(rpcs_ptr) if rpcs_ptr else None,
                                          DEVICE_PTRS, C.c_void_p(stream) if stream else None), "ovs_route_batch")

    def findNode(self, node, keys, numRedundantNodes: int, numSiblings: int, max_out: int = 16):
        keys = keys_array(keys)
        node = np.ascontiguousarray(node, dtype=np.uint32)
        n = len(keys)
        nodes = np.empty((n, max_out), dtype=np.uint32)
        cnt = np.empty(n, dtype=np.uint8)
        sib = np.empty(n, dtype=np.uint8)
        self._chk(self._L.ovs_find_node_batch(self._h, _ptr(node), _ptr(keys), n, numRedundantNodes, numSiblings,
                                              _ptr(nodes), max_out, _ptr(cnt), _ptr(sib), 0, None),
                  "ovs_find_node_batch")
        return nodes, cnt, sib

    def isSiblingFor(self, node, keys, numSiblings: int = 1) -> np.ndarray:
        _, _, sib = self.findNode(node, keys, 1, numSiblings, max_out=1)
        return sib.astype(bool)

    def delay_ns(self, a, b, nbytes) -> np.ndarray:
        a = np.ascontiguousarray(a, dtype=np.uint32)
        b = np.ascontiguousarray(b, dtype=np.uint32)
        nbytes = np.ascontiguousarray(nbytes, dtype=np.int32)
        out = np.empty(len(a), dtype=np.int64)
        self._chk(self._L.ovs_delay_batch(self._h, _ptr(a), _ptr(b), _ptr(nbytes), len(a), _ptr(out), 0, None),
                  "ovs_delay_batch")
        return out

    def sync(self):
        self._chk(self._L.ovs_sync(self._h), "ovs_sync")

    # -- KBRTestApp statistics
    def kbrtest_stats(self, result: dict | np.ndarray, keys, src, measured_time_s: float,
                      lookupNodeIds: bool = True) -> KbrTestStats:
        """Reduce lookup() results to the KBRTestApp one-way statistics on the device."""
        if isinstance(result, dict):
            out = np.empty(len(result["responsible"]), dtype=ROUTE_OUT_DTYPE)
            for f in ROUTE_OUT_DTYPE.names:
                out[f] = result[f]
        else:
            out = np.ascontiguousarray(result, dtype=ROUTE_OUT_DTYPE)
        keys = keys_array(keys)
        src = np.ascontiguousarray(src, dtype=np.uint32)
        if not (len(out) == len(keys) == len(src)):
            raise ValueError("result, keys and src differ in length")
        st = KbrTestStats()
        self._chk(self._L.ovs_kbrtest_stats_batch(self._h, _ptr(out), _ptr(keys), _ptr(src), len(out),
                                                  float(measured_time_s), int(bool(lookupNodeIds)), C.byref(st),
                                                  0, None), "ovs_kbrtest_stats_batch")
        return st

    def kbrtest_lookup_stats(self, result: dict, keys, src, measured_time_s: float, lookupNodeIds: bool = True,
                             failureLatency: float = 10.0) -> KbrTestLookupStats:
        """Reduce lookupCall() results to the KBRTestApp lookup-test statistics on the device."""
        out = np.empty(len(result["hops"]), dtype=LOOKUP_OUT_DTYPE)
        for f in LOOKUP_OUT_DTYPE.names:
            out[f] = result[f]
        sib = np.ascontiguousarray(result["siblings"], dtype=np.uint32)
        keys = keys_array(keys)
        src = np.ascontiguousarray(src, dtype=np.uint32)
        st = KbrTestLookupStats()
        self._chk(self._L.ovs_kbrtest_lookup_stats_batch(self._h, _ptr(out), _ptr(sib), sib.shape[1], _ptr(keys),
                                                         _ptr(src), len(out), float(measured_time_s),
                                                         int(bool(lookupNodeIds)), float(failureLatency),
                                                         C.byref(st), 0, None), "ovs_kbrtest_lookup_stats_batch")
        return st

    def kbrtest_stats_device(self, out_ptr: int, keys_ptr: int, src_ptr: int, n: int, measured_time_s: float,
                             lookupNodeIds: bool = True, stream: int | None = None) -> KbrTestStats:
        """Same as kbrtest_stats for a device-resident batch (synchronises `stream`)."""
        st = KbrTestStats()
        self._chk(self._L.ovs_kbrtest_stats_batch(self._h, C.c_void_p(out_ptr), C.c_void_p(keys_ptr),
                                                  C.c_void_p(src_ptr), n, float(measured_time_s),
                                                  int(bool(lookupNodeIds)), C.byref(st), DEVICE_PTRS,
                                                  C.c_void_p(stream) if stream else None),
                  "ovs_kbrtest_stats_batch")
        return st


@dataclass
class Network:
    """A generated overlay population: sorted unique ids + SimpleUnderlay coordinates."""

    ids: np.ndarray   # (n,5) uint32
    xy: np.ndarray    # (n,2) float64

    @property
    def n(self) -> int:
        return len(self.ids)
