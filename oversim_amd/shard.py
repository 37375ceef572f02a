"""Multi-GPU Chord: the sorted ring cut into contiguous arcs, one per rank, with
lookups handed between ranks every hop round by an all-to-allv.

One process per GPU (torch.distributed; backend "nccl" is RCCL on ROCm, the
exchange runs over xGMI).  Node keys and coordinates are replicated on every
rank, finger rows exist only for the rank's own arc, so a lookup is forwarded
to the rank that owns its next responder -- the message a FindNodeCall would be
in OverSim (BaseOverlay.cc:1841-1915).  Per round:

  1. ovs_shard_step advances every inbound record while its responder is
     local; a hand-off is appended by the kernel to the send segment of its
     destination rank (no grouping pass), finished lookups to the done buffer;
  2. one all-gather of the per-destination counts gives every rank the whole
     count matrix (sizes of the all-to-allv and the termination test) -- the
     round's only host synchronisation;
  3. one all-to-allv moves the records (48 B per lookup): grouped point-to-point
     sends straight out of the kernel's destination segments into one receive
     buffer (no packing copy).

The lookups of a rank are split into cohorts (default 2), each with its own HIP
stream, send segments and counters.  A cohort's kernel, count gather, host wait
and exchange are ordered on its own stream only, so the exchange of one cohort
runs while the kernel of the other computes.

The orchestration is independent of the stepper (the HIP kernel here, a CPU
test double in tests/) and of the exchange (torch.distributed, or an in-process
emulation of W shards on one device).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from .kbr import DEVICE_PTRS, LOOKUP_OUT_DTYPE, KbrEngine, Params, lib

REC_DTYPE = np.dtype([("key", "<u4", 5), ("src", "<u4"), ("cur", "<u4"), ("qid", "<u4"), ("t_ns", "<i8"),
                      ("hops", "<u2"), ("local", "u1"), ("pad", "u1", 5)])
DONE_DTYPE = np.dtype([("qid", "<u4"), ("pad", "<u4"), ("responsible", "<u4"), ("hops", "<u2"), ("status", "u1"),
                       ("one_way_hops", "u1"), ("latency_ns", "<i8")])
assert REC_DTYPE.itemsize == 48 and DONE_DTYPE.itemsize == 24
REC_BYTES, DONE_BYTES = 48, 24


def arc_bounds(n_total: int, world: int) -> list[int]:
    """Contiguous arcs of the sorted ID array, as equal as possible."""
    return [r * n_total // world for r in range(world + 1)]


def prefix_bounds(ids: np.ndarray, world: int) -> list[int]:
    """Arcs cut at key prefixes (the XOR-prefix partition of SURVEY §8e): arc r holds the IDs whose top
    bits lie in [r * 2^160 / W, (r + 1) * 2^160 / W) -- for W a power of two exactly the IDs sharing
    their top log2(W) bits.  Bounds as indices into the sorted ID array."""
    ids = np.ascontiguousarray(ids, dtype=np.uint32).reshape(-1, 5)
    top = (ids[:, 4].astype(np.uint64) << np.uint64(32)) | ids[:, 3].astype(np.uint64)   # the top 64 bits
    cuts = [int(np.searchsorted(top, np.uint64((r << 64) // world), side="left")) for r in range(1, world)]
    return [0] + cuts + [len(ids)]


def default_top_levels(world: int) -> int:
    """Replicated top finger levels for W arcs: the log2(W) levels whose jumps span arcs, plus 3 more
    levels after which a lookup is within 2^(157 - log2 W) of its key, so it crosses to another arc
    about once (at the boundary of its key's arc with probability ~1/8).  64 B per node and level."""
    if world <= 1:
        return 0
    return min(32, int(np.ceil(np.log2(world))) + 3)


# ---------------------------------------------------------------------------
# steppers

class FreshBatch:
    """A batch's first-round inbox: its keys and sources, not yet records (GpuShardStepper.first_batch)."""

    def __init__(self, keys, src, qid_base: int):
        self.keys, self.src, self.qid_base = keys, src, int(qid_base)
        self.shape = (int(keys.shape[0]), REC_BYTES)
        self.device = keys.device


class GpuShardStepper:
    """One rank's arc on one device: owns the engine context and the device buffers."""

    def __init__(self, ids: np.ndarray, xy: np.ndarray, bounds: list[int], rank: int, device, stream=None,
                 capacity: int = 1 << 20, params: Params | None = None, lookup_siblings: int | None = None,
                 top_levels: int | None = None):
        """lookup_siblings: route KBRTestApp LookupCalls with that many siblings (-1 = successorListSize;
        ovs_shard_step_lookup) instead of one-way messages; finish them with lookup_finish().
        top_levels: replicate that many top finger levels of every node (ovs_chord_shard_replicate;
        None = default_top_levels(world)), so a lookup's long first hops are decided at home."""
        import torch
        self.lookup_siblings = lookup_siblings
        self.torch = torch
        self.dev = device
        self.stream = stream
        self.rank, self.bounds, self.world = rank, [int(b) for b in bounds], len(bounds) - 1
        self.eng = KbrEngine(device.index if device.index is not None else 0)
        self.eng.set_params(params or Params.chord())
        ids = np.ascontiguousarray(ids, dtype=np.uint32)
        xy = np.ascontiguousarray(xy, dtype=np.float64)
        st = lib().ovs_chord_load_shard(self.eng._h, ids.ctypes.data_as(C.c_void_p), len(ids),
                                        xy.ctypes.data_as(C.c_void_p), self.bounds[rank], self.bounds[rank + 1], 0)
        self.eng._chk(st, "ovs_chord_load_shard")
        self.top_levels = default_top_levels(self.world) if top_levels is None else int(top_levels)
        if self.top_levels:
            self.eng._chk(lib().ovs_chord_shard_replicate(self.eng._h, self.top_levels), "ovs_chord_shard_replicate")
        self.n_total = len(ids)
        self._lo = (C.c_uint64 * (self.world + 1))(*self.bounds)
        self._cap = {}
        self._out = {}
        self._cnt = {}
        self._ev = {}
        self._timed = {}
        self._streams = []
        self._ensure(0, capacity)
        self.done_count = torch.zeros(1, dtype=torch.int64, device=device)
        self.done = torch.empty((max(capacity, 1), DONE_BYTES), dtype=torch.uint8, device=device)
        self.done_cap = max(capacity, 1)
        self.timing = False
        self.kernel_ms = 0.0

    def _ensure(self, cohort: int, cap: int):
        if cap <= self._cap.get(cohort, 0):
            return
        self._cap[cohort] = cap
        # one send segment of `cap` records per destination rank
        self._out[cohort] = self.torch.empty((self.world, cap, REC_BYTES), dtype=self.torch.uint8, device=self.dev)
        if cohort not in self._cnt:
            self._cnt[cohort] = self.torch.zeros(self.world, dtype=self.torch.int64, device=self.dev)
            self._ev[cohort] = (self.torch.cuda.Event(enable_timing=True), self.torch.cuda.Event(enable_timing=True))

    @property
    def cap(self) -> int:
        return self._cap[0]

    def _s(self):
        # every kernel runs on torch's current stream (the cohort's stream inside cohort()), so
        # the torch ops around it (counter resets, the collectives) are ordered with it
        return C.c_void_p(self.torch.cuda.current_stream(self.dev).cuda_stream)

    def begin_cohorts(self, n: int):
        """n cohort streams, each ordered after the work queued so far (the inputs)."""
        torch = self.torch
        while len(self._streams) < n:
            self._streams.append(torch.cuda.Stream(self.dev))
        cur = torch.cuda.current_stream(self.dev)
        for st in self._streams[:n]:
            st.wait_stream(cur)
        self._ncoh = n

    def end_cohorts(self):
        cur = self.torch.cuda.current_stream(self.dev)
        for st in self._streams[:getattr(self, "_ncoh", 0)]:
            cur.wait_stream(st)

    def cohort(self, c: int):
        """Context in which cohort c's kernels and collectives are issued (its own stream)."""
        return self.torch.cuda.stream(self._streams[c])

    def reset(self, capacity: int):
        self.done_count.zero_()
        if capacity > self.done_cap:
            self.done = self.torch.empty((capacity, DONE_BYTES), dtype=self.torch.uint8, device=self.dev)
            self.done_cap = capacity

    def make_records(self, keys_t, src_t, qid_base: int):
        n = keys_t.shape[0]
        recs = self.torch.empty((n, REC_BYTES), dtype=self.torch.uint8, device=self.dev)
        st = lib().ovs_shard_make_records(self.eng._h, C.c_void_p(keys_t.data_ptr()), C.c_void_p(src_t.data_ptr()),
                                          n, qid_base, C.c_void_p(recs.data_ptr()), self._s())
        self.eng._chk(st, "ovs_shard_make_records")
        return recs

    def first_batch(self, keys_t, src_t, qid_base: int):
        """A batch's first-round inbox without records: step() runs it through ovs_shard_step_keys,
        which starts every lookup from its key and source (no 48 B record written and read back)."""
        return FreshBatch(keys_t, src_t, qid_base)

    def step(self, inbox, cohort: int = 0):
        """One round of a cohort; returns (send segments [world, cap, 48], per-destination counts
        on the device).  The segments stay valid until the cohort's next step."""
        n_in = inbox.shape[0]
        self._ensure(cohort, n_in)
        out, cnt = self._out[cohort], self._cnt[cohort]
        cnt.zero_()
        if self.timing:
            self._ev[cohort][0].record()
        tail = (C.c_void_p(out.data_ptr()), self._cap[cohort], C.c_void_p(cnt.data_ptr()),
                C.c_void_p(self.done.data_ptr()), self.done_cap, C.c_void_p(self.done_count.data_ptr()), self._lo,
                self.world, self._s())
        if isinstance(inbox, FreshBatch):
            ns = 0 if self.lookup_siblings is None else self.lookup_siblings
            self.eng._chk(lib().ovs_shard_step_keys(self.eng._h, ns, C.c_void_p(inbox.keys.data_ptr()),
                                                    C.c_void_p(inbox.src.data_ptr()), n_in, inbox.qid_base, *tail),
                          "ovs_shard_step_keys")
            if self.timing:
                self._ev[cohort][1].record()
                self._timed[cohort] = True
            return out, cnt
        args = (C.c_void_p(inbox.data_ptr()), n_in) + tail
        if self.lookup_siblings is None:
            self.eng._chk(lib().ovs_shard_step(self.eng._h, *args), "ovs_shard_step")
        else:
            self.eng._chk(lib().ovs_shard_step_lookup(self.eng._h, self.lookup_siblings, *args), "ovs_shard_step_lookup")
        if self.timing:
            self._ev[cohort][1].record()
            self._timed[cohort] = True
        return out, cnt

    def collect_timing(self, cohort: int = 0):
        """Add the cohort's last step kernel time (call after its host synchronisation)."""
        if self.timing and self._timed.get(cohort):
            e0, e1 = self._ev[cohort]
            e1.synchronize()
            self.kernel_ms += e0.elapsed_time(e1)
            self._timed[cohort] = False

    def finished(self):
        k = int(self.done_count.item())
        if k > self.done_cap:
            raise RuntimeError("done buffer overflow")
        return self.done[:k]

    def lookup_finish(self, done):
        """LookupResponses of finished LookupCall records (ovs_shard_lookup_finish): (qid, ovs_lookup_out
        records, siblings (n, numSiblings)) as numpy arrays, in the records' order."""
        torch = self.torch
        ns = self.lookup_siblings if self.lookup_siblings and self.lookup_siblings > 0 else \
            self.eng.get_params().successorListSize
        n = done.shape[0]
        out = torch.empty((max(n, 1), 16), dtype=torch.uint8, device=self.dev)
        sib = torch.empty((max(n, 1), ns), dtype=torch.int32, device=self.dev)
        st = lib().ovs_shard_lookup_finish(self.eng._h, C.c_void_p(done.data_ptr()), n, ns, C.c_void_p(out.data_ptr()),
                                           C.c_void_p(sib.data_ptr()), self._s())
        self.eng._chk(st, "ovs_shard_lookup_finish")
        torch.cuda.synchronize(self.dev)
        recs = done_to_numpy(done)
        lo = out[:n].cpu().numpy().reshape(-1).view(LOOKUP_OUT_DTYPE)
        return recs["qid"].copy(), lo, sib[:n].cpu().numpy().view(np.uint32)


for _name, _args in {
    "ovs_chord_load_shard": [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64, C.c_uint64, C.c_uint32],
    "ovs_chord_shard_replicate": [C.c_void_p, C.c_int32],
    "ovs_shard_make_records": [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32, C.c_void_p, C.c_void_p],
    "ovs_shard_step": [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64, C.c_void_p,
                       C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p],
    "ovs_shard_step_lookup": [C.c_void_p, C.c_int32, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64, C.c_void_p,
                              C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p],
    "ovs_shard_lookup_finish": [C.c_void_p, C.c_void_p, C.c_uint64, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p],
    "ovs_shard_step_keys": [C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32, C.c_void_p,
                            C.c_uint64, C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_uint32,
                            C.c_void_p],
    "ovs_kad_load_shard": [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64, C.c_uint64, C.c_uint32],
    "ovs_kad_shard_begin": [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32, C.c_void_p],
    "ovs_kad_shard_begin_lookup": [C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32,
                                   C.c_void_p, C.c_void_p],
    "ovs_kad_shard_step": [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p,
                           C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p],
    "ovs_kad_shard_serve": [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p],
    "ovs_kad_shard_deliver": [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p],
    "ovs_kad_shard_errors": [C.c_void_p, C.c_void_p],
    "ovs_kad_shard_resp_bytes": [C.c_void_p],
    "ovs_kad_shard_replicate": [C.c_void_p, C.c_int32],
    "ovs_kad_shard_mig_step": [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p,
                               C.c_uint64, C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_uint32,
                               C.c_void_p],
    "ovs_rccl_unique_id": [C.c_void_p],
    "ovs_exchange_rccl_create": [C.c_int, C.c_uint32, C.c_uint32, C.c_void_p, C.c_void_p],
    "ovs_exchange_local_create": [C.c_uint32, C.c_void_p],
    "ovs_shard_route_batch": [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p, C.c_uint64,
                              C.c_uint32, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p],
    "ovs_kad_shard_route_batch": [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p, C.c_uint64,
                                  C.c_uint32, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p],
}.items():
    _f = getattr(lib(), _name)
    _f.argtypes = _args
    _f.restype = C.c_int
lib().ovs_exchange_destroy.argtypes = [C.c_void_p]
lib().ovs_exchange_destroy.restype = None
lib().ovs_exchange_last_error.argtypes = []
lib().ovs_exchange_last_error.restype = C.c_char_p
lib().ovs_exchange_stage.argtypes = [C.POINTER(C.c_uint32)]
lib().ovs_exchange_stage.restype = C.c_char_p
lib().ovs_chord_shard_levels.argtypes = [C.c_void_p]
lib().ovs_chord_shard_levels.restype = C.c_int32
lib().ovs_kad_shard_levels.argtypes = [C.c_void_p]
lib().ovs_kad_shard_levels.restype = C.c_int32
lib().ovs_kad_shard_rec_bytes.argtypes = [C.c_void_p]
lib().ovs_kad_shard_rec_bytes.restype = C.c_int32


# ---------------------------------------------------------------------------
# the round loop behind the C ABI (ovs_shard_route_batch / ovs_kad_shard_route_batch) and its exchanges

ALLGATHER_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_int64), C.c_uint32, C.POINTER(C.c_int64))
ALLTOALLV_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_uint64), C.c_void_p,
                           C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.c_uint32, C.c_void_p)
ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_int64), C.c_uint32)
DESTROY_FN = C.CFUNCTYPE(None, C.c_void_p)


class Exchange(C.Structure):
    """ovs_exchange (include/ovs_kbr.h): the collective callbacks the native round loop runs over."""
    _fields_ = [("user", C.c_void_p), ("rank", C.c_uint32), ("world", C.c_uint32),
                ("allgather_i64", ALLGATHER_FN), ("alltoallv", ALLTOALLV_FN),
                ("allreduce_sum_i64", ALLREDUCE_FN), ("destroy", DESTROY_FN)]


class RouteStats(C.Structure):
    """ovs_shard_route_stats."""
    _fields_ = [("rounds", C.c_uint32), ("cohorts", C.c_uint32), ("sent", C.c_uint64), ("sent_bytes", C.c_uint64),
                ("done", C.c_uint64), ("step_ms", C.c_double), ("exchange_ms", C.c_double), ("total_ms", C.c_double)]

    def as_dict(self) -> dict:
        return {f: getattr(self, f) for f, _ in self._fields_}


def _exchange_error(what: str, st: int):
    msg = lib().ovs_exchange_last_error()
    raise RuntimeError(f"{what}: status {st}: {msg.decode() if msg else ''}")


def rccl_exchange(rank: int, world: int, device_index: int, unique_id: bytes) -> Exchange:
    """The library's RCCL exchange (ovs_exchange_rccl_create); unique_id from rccl_unique_id() on rank 0."""
    ex = Exchange()
    buf = C.create_string_buffer(bytes(unique_id), 128)
    st = lib().ovs_exchange_rccl_create(device_index, rank, world, buf, C.byref(ex))
    if st != 0:
        _exchange_error("ovs_exchange_rccl_create", st)
    return ex


def rccl_unique_id() -> bytes:
    buf = C.create_string_buffer(128)
    st = lib().ovs_rccl_unique_id(buf)
    if st != 0:
        _exchange_error("ovs_rccl_unique_id", st)
    return buf.raw


def rccl_exchange_from_torch(device_index: int) -> Exchange:
    """An RCCL exchange for every rank of torch.distributed's default group (rank 0's unique id
    broadcast through the group)."""
    import torch.distributed as dist
    obj = [rccl_unique_id() if dist.get_rank() == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    return rccl_exchange(dist.get_rank(), dist.get_world_size(), device_index, obj[0])


def local_exchanges(world: int) -> list:
    """W in-process ranks (threads): one exchange per rank (ovs_exchange_local_create)."""
    arr = (Exchange * world)()
    st = lib().ovs_exchange_local_create(world, arr)
    if st != 0:
        _exchange_error("ovs_exchange_local_create", st)
    return [arr[r] for r in range(world)]


def destroy_exchange(ex: Exchange):
    lib().ovs_exchange_destroy(C.byref(ex))


class _DevBytes:
    """A device byte range as a torch tensor (__cuda_array_interface__)."""

    def __init__(self, ptr: int, nbytes: int):
        self.__cuda_array_interface__ = {"shape": (int(nbytes),), "typestr": "|u1", "data": (int(ptr), False),
                                         "version": 2, "strides": None}


class CallbackExchange:
    """An ovs_exchange whose callbacks run torch.distributed collectives (gloo on CPU tensors): the
    native round loop over a Python-side process group -- how the tests drive it with gloo, and how
    a caller could plug any transport in."""

    def __init__(self, device, group=None):
        import torch
        import torch.distributed as dist
        self.torch, self.dist, self.group, self.dev = torch, dist, group, device
        self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)
        self._cb = (ALLGATHER_FN(self._allgather), ALLTOALLV_FN(self._alltoallv), ALLREDUCE_FN(self._allreduce),
                    DESTROY_FN())
        self.ex = Exchange(None, self.rank, self.world, *self._cb)
        self.ex._owner = self          # keeps the callbacks alive with the table
        self.error = None

    def _guard(self, f, *a):
        try:
            f(*a)
            return 0
        except Exception as e:       # a Python exception must not unwind through C frames
            import sys
            import traceback
            self.error = e
            traceback.print_exc(file=sys.stderr)
            return 1

    def _allgather(self, user, send, n, recv):
        def run():
            torch = self.torch
            t = torch.tensor([send[i] for i in range(n)], dtype=torch.int64)
            parts = [torch.empty_like(t) for _ in range(self.world)]
            self.dist.all_gather(parts, t, group=self.group)
            flat = torch.cat(parts).tolist()
            for i, v in enumerate(flat):
                recv[i] = v
        return self._guard(run)

    def _allreduce(self, user, vals, n):
        def run():
            t = self.torch.tensor([vals[i] for i in range(n)], dtype=self.torch.int64)
            self.dist.all_reduce(t, group=self.group)
            for i, v in enumerate(t.tolist()):
                vals[i] = v
        return self._guard(run)

    def _alltoallv(self, user, send, send_rows, recv, recv_off, recv_rows, row_bytes, stream):
        def run():
            torch, dist = self.torch, self.dist
            # the segments are complete (stream NULL: the device's default stream)
            if stream:
                torch.cuda.ExternalStream(stream, device=self.dev).synchronize()
            else:
                torch.cuda.synchronize(self.dev)
            ops, host_recv = [], {}
            for r in range(self.world):
                ns, nr = int(send_rows[r]) * row_bytes, int(recv_rows[r]) * row_bytes
                if r == self.rank:
                    if nr:
                        dst = torch.as_tensor(_DevBytes(recv + int(recv_off[r]) * row_bytes, nr), device=self.dev)
                        dst.copy_(torch.as_tensor(_DevBytes(send[r], ns), device=self.dev))
                    continue
                if ns:
                    ops.append(dist.P2POp(dist.isend, torch.as_tensor(_DevBytes(send[r], ns), device=self.dev).cpu(),
                                          r, group=self.group))
                if nr:
                    host_recv[r] = torch.empty(nr, dtype=torch.uint8)
                    ops.append(dist.P2POp(dist.irecv, host_recv[r], r, group=self.group))
            if ops:
                for w in dist.batch_isend_irecv(ops):
                    w.wait()
            for r, t in host_recv.items():
                torch.as_tensor(_DevBytes(recv + int(recv_off[r]) * row_bytes, t.numel()), device=self.dev).copy_(t)
            torch.cuda.synchronize(self.dev)
        return self._guard(run)


def exchange_sum(ex: Exchange, values) -> list:
    """Element-wise sum of int64 values over the exchange's ranks (its allreduce callback): a
    collective -- every rank calls it."""
    arr = (C.c_int64 * len(values))(*[int(v) for v in values])
    if ex.allreduce_sum_i64(ex.user, arr, len(values)) != 0:
        raise RuntimeError(f"exchange allreduce failed: {lib().ovs_exchange_last_error().decode()}")
    return list(arr)


def native_route(stepper, ex: Exchange, keys_t, src_t, qid_base: int, cohorts: int = 2, num_siblings: int = 0,
                 stream=None, done_cap: int | None = None) -> tuple:
    """Route this rank's Chord batch through ovs_shard_route_batch (the round loop in C++);
    returns (done records [k, 24] uint8 on the device, RouteStats).  done_cap: at most the stepper's
    (tests shrink it to provoke a one-rank failure)."""
    torch = stepper.torch
    n = int(keys_t.shape[0])
    bounds = (C.c_uint64 * (stepper.world + 1))(*stepper.bounds)
    nd = C.c_uint64(0)
    stats = RouteStats()
    s = stream if stream is not None else torch.cuda.current_stream(stepper.dev).cuda_stream
    cap = stepper.done_cap if done_cap is None else min(int(done_cap), stepper.done_cap)
    st = lib().ovs_shard_route_batch(stepper.eng._h, C.byref(ex), bounds, num_siblings, C.c_void_p(keys_t.data_ptr()),
                                     C.c_void_p(src_t.data_ptr()), n, qid_base, C.c_void_p(stepper.done.data_ptr()),
                                     cap, C.byref(nd), cohorts, C.byref(stats), C.c_void_p(s))
    if st != 0 and isinstance(getattr(ex, "_owner", None), CallbackExchange) and ex._owner.error:
        raise RuntimeError(f"exchange callback failed: {ex._owner.error!r}")
    stepper.eng._chk(st, "ovs_shard_route_batch")
    return stepper.done[:nd.value], stats


def native_kad_route(stepper, ex: Exchange, keys_t, src_t, qid_base: int, num_siblings: int = -2,
                     stream=None, done_cap: int | None = None) -> tuple:
    """Route this rank's Kademlia batch through ovs_kad_shard_route_batch; returns (done [n, 24], RouteStats)."""
    torch = stepper.torch
    n = int(keys_t.shape[0])
    bounds = (C.c_uint64 * (stepper.world + 1))(*stepper.bounds)
    stepper.n = n
    # migrating lookups (replicated top buckets, one-way routes) finish on any rank: room for every
    # lookup of the batch, summed over the ranks (batches may differ in size)
    migrate = num_siblings < -1 and getattr(stepper, "top_levels", 0)
    rows = exchange_sum(ex, [n])[0] if migrate else n
    if getattr(stepper, "done", None) is None or stepper.done.shape[0] < max(rows, 1):
        stepper.done = torch.empty((max(rows, 1), DONE_BYTES), dtype=torch.uint8, device=stepper.dev)
    sib = None
    if num_siblings >= -1:
        ns = num_siblings if num_siblings >= 0 else stepper.params.s
        stepper.sib = torch.empty((max(n, 1), max(ns, 1)), dtype=torch.int32, device=stepper.dev)
        sib = C.c_void_p(stepper.sib.data_ptr())
        stepper.qid_base = qid_base
    nd = C.c_uint64(0)
    stats = RouteStats()
    s = stream if stream is not None else torch.cuda.current_stream(stepper.dev).cuda_stream
    st = lib().ovs_kad_shard_route_batch(stepper.eng._h, C.byref(ex), bounds, num_siblings,
                                         C.c_void_p(keys_t.data_ptr()), C.c_void_p(src_t.data_ptr()), n, qid_base,
                                         C.c_void_p(stepper.done.data_ptr()),
                                         stepper.done.shape[0] if done_cap is None else min(int(done_cap), stepper.done.shape[0]),
                                         C.byref(nd), sib,
                                         C.byref(stats), C.c_void_p(s))
    if st != 0 and isinstance(getattr(ex, "_owner", None), CallbackExchange) and ex._owner.error:
        raise RuntimeError(f"exchange callback failed: {ex._owner.error!r}")
    stepper.eng._chk(st, "ovs_kad_shard_route_batch")
    return stepper.done[:nd.value], stats


# ---------------------------------------------------------------------------
# exchanges of the Python round loop (route_sharded / route_kad_sharded)

class TorchExchange:
    """all-to-allv of fixed-size records over torch.distributed (RCCL on GPUs, gloo on CPU)."""

    def __init__(self, world: int, device, group=None):
        import torch
        import torch.distributed as dist
        self.torch, self.dist, self.world, self.group = torch, dist, world, group
        self.rank = dist.get_rank(group)
        self.comm_dev = device   # tensors handed to the collective live here

    def count_matrix(self, counts) -> np.ndarray:
        """All-gather every rank's per-destination counts: M[s, d] = records rank s sends to d."""
        return self.count_matrix_async(counts)()

    def count_matrix_async(self, counts):
        """Start the count all-gather on the current stream; returns a callable that waits for
        it (and only for the work queued on this stream) and gives the matrix."""
        torch = self.torch
        c = counts.to(self.comm_dev, dtype=torch.int64).reshape(-1)
        parts = [torch.empty_like(c) for _ in range(self.world)]
        self.dist.all_gather(parts, c, group=self.group)
        M = torch.stack(parts)
        if M.device.type != "cuda":
            return lambda: M.numpy()
        host = torch.empty(M.shape, dtype=torch.int64, pin_memory=True)
        host.copy_(M, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()

        def wait():
            ev.synchronize()
            return host.numpy()
        return wait

    # rows per point-to-point message: a big all-to-allv goes out in pieces of at most 256 MB
    # (both sides cut a transfer identically, and messages between two ranks match in order)
    CHUNK_BYTES = 256 << 20

    def _p2p(self, ops, t, peer, send: bool):
        dist = self.dist
        step = max(1, self.CHUNK_BYTES // max(1, t.shape[1] if t.dim() > 1 else 1))
        for a in range(0, t.shape[0], step):
            ops.append(dist.P2POp(dist.isend if send else dist.irecv, t[a:a + step], peer, group=self.group))

    def _run(self, ops):
        if ops:
            for w in self.dist.batch_isend_irecv(ops):
                w.wait()

    def segments(self, segs, scl, rcl, row_bytes: int):
        """all-to-allv of fixed-size records from per-destination segments (segs[d][:scl[d]])
        into one receive buffer ordered by source rank: grouped point-to-point sends out of
        the segments, so nothing is packed first; this rank's own share is a device copy."""
        torch = self.torch
        # 0xFF sentinel: a row the exchange never wrote reads as an impossible record (node / cur /
        # tag 0xFFFFFFFF), which the consuming kernel counts as an error instead of using
        recv = torch.full((sum(rcl), row_bytes), 0xFF, dtype=torch.uint8, device=self.comm_dev)
        ops, off = [], 0
        for r in range(self.world):
            if rcl[r] and r != self.rank:
                self._p2p(ops, recv[off:off + rcl[r]], r, send=False)
            elif rcl[r]:
                recv[off:off + rcl[r]].copy_(segs[r][:rcl[r]])
            off += rcl[r]
        for d in range(self.world):
            if scl[d] and d != self.rank:
                self._p2p(ops, segs[d][:scl[d]].to(self.comm_dev), d, send=True)
        self._run(ops)
        return recv

    def counts(self, send_counts):
        """Exchange per-destination counts; returns (send counts, receive counts) as lists."""
        torch, dist = self.torch, self.dist
        sc = send_counts.to(self.comm_dev, dtype=torch.int64)
        rc = torch.empty_like(sc)
        dist.all_to_all_single(rc, sc, group=self.group)
        return sc.tolist(), rc.tolist()

    def records(self, send, scl, rcl):
        """all-to-allv of rows of `send` (uint8, one record per row, grouped by destination rank)
        with explicit splits: point-to-point pieces to the other ranks, a device copy of this
        rank's own share (one RCCL message above 2^30 bytes delivers only its first half: DESIGN.md §6)."""
        torch = self.torch
        send = send.to(self.comm_dev)
        recv = torch.full((sum(rcl), send.shape[1]), 0xFF, dtype=torch.uint8, device=self.comm_dev)   # sentinel
        ops = []
        so = np.concatenate([[0], np.cumsum(scl)]).astype(np.int64)
        ro = np.concatenate([[0], np.cumsum(rcl)]).astype(np.int64)
        for r in range(self.world):
            if r == self.rank:
                if rcl[r]:
                    recv[ro[r]:ro[r + 1]].copy_(send[so[r]:so[r + 1]])
                continue
            if rcl[r]:
                self._p2p(ops, recv[ro[r]:ro[r + 1]], r, send=False)
            if scl[r]:
                self._p2p(ops, send[so[r]:so[r + 1]], r, send=True)
        self._run(ops)
        return recv

    def total(self, x: int) -> int:
        t = self.torch.tensor([x], dtype=self.torch.int64, device=self.comm_dev)
        self.dist.all_reduce(t, group=self.group)
        return int(t.item())

    def exchange(self, send, send_counts):
        scl, rcl = self.counts(send_counts)
        if self.total(sum(scl)) == 0:
            return None
        return self.records(send, scl, rcl)


def route_sharded(stepper, exchange, keys_t, src_t, qid_base: int, max_rounds: int = 10_000, cohorts: int = 2,
                  min_split: int = 2048):
    """Route one batch of lookups originating on this rank; returns (done records, rounds).

    The batch is split into `cohorts` contiguous cohorts (one if the stepper has no cohort
    support or the batch is small).  Every round first issues the step kernel of each live
    cohort (each on its own stream; the persistent grids run one after the other), then per
    cohort its count gather, the host wait for it and its exchange.  The collectives share
    one communicator stream in issue order (gather 0, exchange 0, gather 1, exchange 1), so
    cohort 0's exchange is in flight while cohort 1's kernel still runs, and cohort 1's while
    cohort 0's next kernel runs.  Every rank takes the same decisions from the same gathered
    matrices, so the collectives match across ranks."""
    n = int(keys_t.shape[0])
    if not hasattr(stepper, "cohort") or n < min_split * cohorts:
        cohorts = 1
    bounds = [c * n // cohorts for c in range(cohorts + 1)]
    me = exchange.rank
    if hasattr(stepper, "begin_cohorts"):
        stepper.begin_cohorts(cohorts)
    ctx = stepper.cohort if hasattr(stepper, "cohort") else (lambda c: _NoCtx())
    step = (lambda inbox, c: stepper.step(inbox, c)) if hasattr(stepper, "cohort") else (lambda inbox, c: stepper.step(inbox))
    inbox = []
    first = getattr(stepper, "first_batch", stepper.make_records)
    for c in range(cohorts):
        with ctx(c):
            inbox.append(first(keys_t[bounds[c]:bounds[c + 1]], src_t[bounds[c]:bounds[c + 1]], qid_base + bounds[c]))
    live = [True] * cohorts
    rounds = 0
    while any(live):
        rounds += 1
        issued = []
        for c in range(cohorts):
            if live[c]:
                with ctx(c):
                    issued.append((c,) + tuple(step(inbox[c], c)))
        for c, out, counts in issued:
            with ctx(c):
                M = exchange.count_matrix_async(counts)()     # the cohort's round synchronisation
                if hasattr(stepper, "collect_timing"):
                    stepper.collect_timing(c) if hasattr(stepper, "cohort") else stepper.collect_timing()
                if int(M.sum()) == 0:
                    live[c] = False
                    continue
                recv = exchange.segments(out, M[me].tolist(), M[:, me].tolist(), REC_BYTES)
                inbox[c] = recv if recv.device == stepper.dev else recv.to(stepper.dev)
        if rounds > max_rounds:
            raise RuntimeError("sharded routing did not terminate")
    if hasattr(stepper, "end_cohorts"):
        stepper.end_cohorts()
    done = stepper.finished()
    # Chord lookups finish on whichever rank holds them last: the batch is complete when the ranks'
    # finished records add up to their lookups (one small all-reduce per batch)
    check_complete(done, n, "sharded Chord", exchange=exchange)
    return done, rounds


def check_complete(done, n: int, what: str, exchange=None, sentinel: bool = True):
    """No finished record came from an exchange row that was never written (the 0xFF sentinel reads
    as qid 0xFFFFFFFF, status BROKEN), and the finished records match the lookups -- this rank's
    (exchange None: a rank finishes exactly its own lookups) or all ranks' together.  A short
    transfer surfaces here, not as lost lookups.  sentinel = False: the records never travelled
    (Kademlia lookups finish on their home rank; a lost response ends its lookup as a counted
    ovs_kad_shard_errors instead)."""
    k = len(done)
    if sentinel and k and hasattr(done, "dim") and done.dim() == 2:     # device records (test doubles hand lists)
        # the qid word of a sentinel record is 0xFFFFFFFF: one strided compare + any over the qid column
        # (the byte-wise all() over (n, 4) cost 0.3 ms per 10M records)
        if done.shape[1] % 4 == 0 and done.is_contiguous():
            import torch
            sent = int((done.view(torch.int32)[:, 0] == -1).sum().item())
        else:
            sent = int((done[:, :4] == 0xFF).all(dim=1).sum().item())
        if sent:
            raise RuntimeError(f"{what}: {sent} finished records from unwritten or corrupt exchange rows")
    have, want = k, n
    if exchange is not None and hasattr(exchange, "total"):
        have, want = exchange.total(k), exchange.total(n)
    if have != want:
        raise RuntimeError(f"{what}: {have} finished records for {want} lookups")


class _NoCtx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def route_local_shards(steppers, keys_per_shard, src_per_shard, qid_bases, max_rounds: int = 10_000):
    """Single-process emulation of W ranks (e.g. W contexts on one GPU): the exchange is a concatenation."""
    import torch
    W = len(steppers)
    def first(st):      # a stepper that starts from the keys, else the records of make_records
        return st.first_batch if hasattr(st, "first_batch") else st.make_records
    inbox = [first(steppers[r])(keys_per_shard[r], src_per_shard[r], qid_bases[r]) for r in range(W)]
    rounds = 0
    while True:
        rounds += 1
        buckets = [[] for _ in range(W)]
        moved = 0
        for r in range(W):
            out, counts = steppers[r].step(inbox[r])
            row = counts.cpu().tolist()
            if hasattr(steppers[r], "collect_timing"):
                steppers[r].collect_timing()
            for d, k in enumerate(row):
                if k:
                    buckets[d].append(out[d][:k].clone())
                    moved += k
        if moved == 0:
            break
        dev = steppers[0].dev
        rb = getattr(steppers[0], "rec_bytes", REC_BYTES)
        inbox = [torch.cat(b) if b else torch.empty((0, rb), dtype=torch.uint8, device=dev) for b in buckets]
        if rounds > max_rounds:
            raise RuntimeError("sharded routing did not terminate")
    return [s.finished() for s in steppers], rounds


# ---------------------------------------------------------------------------
# Kademlia: lookups stay home, FindNodeCalls are requests to the responder's owner

KAD_REQ_DTYPE = np.dtype([("key", "<u4", 5), ("node", "<u4"), ("tag", "<u4"), ("pad", "<u4")])
KAD_RESP_DTYPE = np.dtype([("tag", "<u4"), ("count", "<u4"), ("nodes", "<u4", 8), ("dist_hi", "<u8", 8)])
# KademliaLarge (k or lookupRedundantNodes above 8): ovs_kad_resp16
KAD_RESP16_DTYPE = np.dtype([("tag", "<u4"), ("count", "<u4"), ("nodes", "<u4", 16), ("dist_hi", "<u8", 16)])
KAD_REQ_BYTES, KAD_RESP_BYTES = KAD_REQ_DTYPE.itemsize, KAD_RESP_DTYPE.itemsize
assert (KAD_REQ_BYTES, KAD_RESP_BYTES, KAD_RESP16_DTYPE.itemsize) == (32, 104, 200)


class KadShardStepper:
    """One rank's arc of a Kademlia network on one device (ovs_kad_load_shard + shard kernels)."""

    def __init__(self, ids: np.ndarray, xy: np.ndarray, bounds: list[int], rank: int, device,
                 params: Params | None = None, lookup_siblings: int | None = None, top_levels: int = 0):
        """lookup_siblings: run KBRTestApp LookupCalls with that many siblings (-1 = s, 0 = exact-key
        lookup; ovs_kad_shard_begin_lookup) instead of one-way routes; results via lookup_results().
        top_levels: replicate the top buckets of every node (ovs_kad_shard_replicate) -- one-way
        routes through the native loop then migrate (KadMigStepper is the Python stepper of that mode)."""
        import torch
        self.torch, self.dev = torch, device
        self.rank, self.bounds, self.world = rank, [int(b) for b in bounds], len(bounds) - 1
        self.eng = KbrEngine(device.index if device.index is not None else 0)
        self.params = params or Params.kademlia()
        self.eng.set_params(self.params)
        self.lookup_siblings = lookup_siblings
        ids = np.ascontiguousarray(ids, dtype=np.uint32)
        xy = np.ascontiguousarray(xy, dtype=np.float64)
        st = lib().ovs_kad_load_shard(self.eng._h, ids.ctypes.data_as(C.c_void_p), len(ids),
                                      xy.ctypes.data_as(C.c_void_p), self.bounds[rank], self.bounds[rank + 1], 0)
        self.eng._chk(st, "ovs_kad_load_shard")
        self.top_levels = int(top_levels)
        if self.top_levels:
            self.eng._chk(lib().ovs_kad_shard_replicate(self.eng._h, self.top_levels), "ovs_kad_shard_replicate")
        self._lo = (C.c_uint64 * (self.world + 1))(*self.bounds)
        # counts[0..world): requests per owner rank, counts[world]: lookups still active, counts[world+1]: done
        self.counts = torch.zeros(self.world + 2, dtype=torch.int64, device=device)
        self.n = 0
        self.served = 0   # FindNodeCalls answered by this rank (requests served)
        self.timing = False
        self.kernel_ms = 0.0
        self._ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        self._timed = False
        # response records: 104 B, or 200 B (ovs_kad_resp16) for KademliaLarge
        self.resp_bytes = int(lib().ovs_kad_shard_resp_bytes(self.eng._h))

    def _s(self):
        return C.c_void_p(self.torch.cuda.current_stream(self.dev).cuda_stream)

    def _p(self, t, off=0):
        return C.c_void_p(t.data_ptr() + off)

    def begin(self, keys_t, src_t, qid_base: int):
        torch = self.torch
        n = keys_t.shape[0]
        self.n = n
        a = self.params.lookupParallelRpcs
        a = a if a <= 4 else 8      # pending-call slots: the K2 instantiation's capacity (kad_pend_slots)
        # one round sends at most alpha requests per lookup (a request occupies a pending slot
        # until its result is delivered at the end of the round): a segment per owner rank
        self.seg_cap = max(n * a, 1)
        self.out = torch.empty((self.world, self.seg_cap, KAD_REQ_BYTES), dtype=torch.uint8, device=self.dev)
        self.done = torch.empty((max(n, 1), DONE_BYTES), dtype=torch.uint8, device=self.dev)
        self.counts.zero_()
        self.qid_base = qid_base
        if self.lookup_siblings is None:
            st = lib().ovs_kad_shard_begin(self.eng._h, self._p(keys_t), self._p(src_t), n, qid_base, self._s())
            self.eng._chk(st, "ovs_kad_shard_begin")
            return
        ns = self.lookup_siblings if self.lookup_siblings >= 0 else self.params.s
        self.sib = torch.empty((max(n, 1), max(ns, 1)), dtype=torch.int32, device=self.dev)
        st = lib().ovs_kad_shard_begin_lookup(self.eng._h, self.lookup_siblings, self._p(keys_t), self._p(src_t), n,
                                              qid_base, self._p(self.sib), self._s())
        self.eng._chk(st, "ovs_kad_shard_begin_lookup")

    def step(self):
        """One round, stream-ordered (no host synchronisation): returns (per-owner request segments
        [world, seg_cap, 32], device counts [world + 2]: requests per owner, active lookups, done)."""
        self.counts[:self.world].zero_()
        if self.timing:
            self._ev[0].record()
        W = self.world
        st = lib().ovs_kad_shard_step(self.eng._h, self._p(self.out), self.seg_cap, self._p(self.counts),
                                      self._p(self.done), self.done.shape[0], self._p(self.counts, 8 * (W + 1)),
                                      self._p(self.counts, 8 * W), self._lo, W, self._s())
        self.eng._chk(st, "ovs_kad_shard_step")
        if self.timing:
            self._ev[1].record()
            self._timed = True
        return self.out, self.counts

    def collect_timing(self):
        """Add the last step kernel's time (call after the round's host synchronisation)."""
        if self.timing and self._timed:
            self._ev[1].synchronize()
            self.kernel_ms += self._ev[0].elapsed_time(self._ev[1])
            self._timed = False

    def serve(self, reqs):
        n = reqs.shape[0]
        self.served += n
        resp = self.torch.empty((n, self.resp_bytes), dtype=self.torch.uint8, device=self.dev)
        if n:
            st = lib().ovs_kad_shard_serve(self.eng._h, self._p(reqs), n, self._p(resp), self._s())
            self.eng._chk(st, "ovs_kad_shard_serve")
        return resp

    def deliver(self, resps):
        if resps.shape[0]:
            st = lib().ovs_kad_shard_deliver(self.eng._h, self._p(resps), resps.shape[0], self._s())
            self.eng._chk(st, "ovs_kad_shard_deliver")

    def errors(self) -> int:
        """ovs_kad_shard_errors: undeliverable responses (mis-routed or lost requests), table reads off
        this arc, and sources off this rank's arc."""
        bad = C.c_uint64(0)
        self.eng._chk(lib().ovs_kad_shard_errors(self.eng._h, C.byref(bad)), "ovs_kad_shard_errors")
        return int(bad.value)

    def finished(self):
        k = int(self.counts[self.world + 1].item())
        if k > self.done.shape[0]:
            raise RuntimeError("done buffer overflow")
        bad = self.errors()
        if bad:
            raise RuntimeError(f"{bad} Kademlia shard errors: responses that could not be delivered (request sent "
                               "to the wrong rank or lost in the exchange), table reads off the arc, or lookups "
                               "whose source lies off this rank's arc")
        return self.done[:k]

    def lookup_results(self, done):
        """LookupCall mode: (qid, ovs_lookup_out records, siblings rows) of finished records, in their order."""
        recs = done_to_numpy(done)
        qid = recs["qid"].copy()
        lo = done[:, 8:24].contiguous().cpu().numpy().reshape(-1).view(LOOKUP_OUT_DTYPE)
        sib = self.sib.cpu().numpy().view(np.uint32)[qid - np.uint32(self.qid_base)]
        return qid, lo, sib


class KadMigStepper:
    """One rank's arc of a Kademlia network whose one-way lookups MIGRATE (ovs_kad_shard_mig_step): the
    stepper interface of GpuShardStepper (first_batch / step / finished), so route_local_shards and
    route_sharded drive it; records are ovs_kad_shard_rec_bytes bytes."""

    def __init__(self, ids: np.ndarray, xy: np.ndarray, bounds: list[int], rank: int, device,
                 params: Params | None = None, top_levels: int = 3, capacity: int = 1 << 16):
        import torch
        self.torch, self.dev = torch, device
        self.rank, self.bounds, self.world = rank, [int(b) for b in bounds], len(bounds) - 1
        self.eng = KbrEngine(device.index if device.index is not None else 0)
        self.params = params or Params.kademlia()
        self.eng.set_params(self.params)
        ids = np.ascontiguousarray(ids, dtype=np.uint32)
        xy = np.ascontiguousarray(xy, dtype=np.float64)
        st = lib().ovs_kad_load_shard(self.eng._h, ids.ctypes.data_as(C.c_void_p), len(ids),
                                      xy.ctypes.data_as(C.c_void_p), self.bounds[rank], self.bounds[rank + 1], 0)
        self.eng._chk(st, "ovs_kad_load_shard")
        self.top_levels = int(top_levels)
        self.eng._chk(lib().ovs_kad_shard_replicate(self.eng._h, self.top_levels), "ovs_kad_shard_replicate")
        self.rec_bytes = int(lib().ovs_kad_shard_rec_bytes(self.eng._h))
        self._lo = (C.c_uint64 * (self.world + 1))(*self.bounds)
        self._cap = 0
        self.cnt = torch.zeros(self.world, dtype=torch.int64, device=device)
        self.done_count = torch.zeros(1, dtype=torch.int64, device=device)
        self.done = torch.empty((max(capacity, 1), DONE_BYTES), dtype=torch.uint8, device=device)
        self.done_cap = max(capacity, 1)
        self.timing = False
        self.kernel_ms = 0.0

    def reset(self, capacity: int):
        self.done_count.zero_()
        if capacity > self.done_cap:
            self.done = self.torch.empty((capacity, DONE_BYTES), dtype=self.torch.uint8, device=self.dev)
            self.done_cap = capacity

    def first_batch(self, keys_t, src_t, qid_base: int):
        return FreshBatch(keys_t, src_t, qid_base)

    def _s(self):
        return C.c_void_p(self.torch.cuda.current_stream(self.dev).cuda_stream)

    def step(self, inbox):
        torch = self.torch
        n_in = inbox.shape[0]
        if n_in > self._cap:
            self._cap = n_in
            self.out = torch.empty((self.world, max(n_in, 1), self.rec_bytes), dtype=torch.uint8, device=self.dev)
        self.cnt.zero_()
        p = lambda t: C.c_void_p(t.data_ptr())
        if isinstance(inbox, FreshBatch):
            st = lib().ovs_kad_shard_mig_step(self.eng._h, None, n_in, p(inbox.keys), p(inbox.src), inbox.qid_base,
                                              p(self.out), self._cap, p(self.cnt), p(self.done), self.done_cap,
                                              p(self.done_count), self._lo, self.world, self._s())
        else:
            st = lib().ovs_kad_shard_mig_step(self.eng._h, p(inbox), n_in, None, None, 0, p(self.out), self._cap,
                                              p(self.cnt), p(self.done), self.done_cap, p(self.done_count), self._lo,
                                              self.world, self._s())
        self.eng._chk(st, "ovs_kad_shard_mig_step")
        return self.out, self.cnt

    def errors(self) -> int:
        bad = C.c_uint64(0)
        self.eng._chk(lib().ovs_kad_shard_errors(self.eng._h, C.byref(bad)), "ovs_kad_shard_errors")
        return int(bad.value)

    def finished(self):
        k = int(self.done_count.item())
        if k > self.done_cap:
            raise RuntimeError("done buffer overflow")
        bad = self.errors()
        if bad:
            raise RuntimeError(f"{bad} Kademlia shard errors (table reads off the arc)")
        return self.done[:k]


def route_kad_sharded(stepper, exchange, keys_t, src_t, qid_base: int, max_rounds: int = 5_000):
    """Route this rank's Kademlia lookups.  Per round: the step kernel, ONE host synchronisation (the
    all-gather of every rank's per-owner request counts and active lookups), then the requests to the
    owners, their findNode answers and the responses back (2 all-to-allv with the splits the matrix
    gives) -- all stream-ordered."""
    stepper.begin(keys_t, src_t, qid_base)
    W, me = exchange.world, exchange.rank
    rounds = 0
    while True:
        rounds += 1
        segs, counts = stepper.step()
        M = exchange.count_matrix_async(counts[:W + 1])()      # M[s, d] requests s -> d, M[s, W] active on s
        if hasattr(stepper, "collect_timing"):
            stepper.collect_timing()
        if int(M.sum()) == 0:
            break
        scl, rcl = M[me, :W].tolist(), M[:W, me].tolist()
        reqs = exchange.segments(segs, scl, rcl, KAD_REQ_BYTES)
        resps = stepper.serve(reqs if reqs.device == stepper.dev else reqs.to(stepper.dev))
        back = exchange.records(resps, rcl, scl)          # reverse splits: back to the requesters
        stepper.deliver(back if back.device == stepper.dev else back.to(stepper.dev))
        if rounds > max_rounds:
            raise RuntimeError(f"sharded Kademlia routing did not terminate: {int(M[:, W].sum())} lookups active, "
                               f"{int(M[:, :W].sum())} requests in round {rounds}")
    done = stepper.finished()
    check_complete(done, int(keys_t.shape[0]), "sharded Kademlia", sentinel=False)
    return done, rounds


def route_kad_local_shards(steppers, keys_per_shard, src_per_shard, qid_bases, max_rounds: int = 100_000):
    """Single-process emulation of W Kademlia ranks (W contexts on one device)."""
    import torch
    W = len(steppers)
    for r in range(W):
        steppers[r].begin(keys_per_shard[r], src_per_shard[r], qid_bases[r])
    rounds = 0
    while True:
        rounds += 1
        segs, rows = [], []
        for r in range(W):
            sg, counts = steppers[r].step()
            segs.append(sg)
            rows.append(counts[:W + 1].cpu().numpy().copy())
        M = np.stack(rows)
        if int(M.sum()) == 0:
            break
        # requests to owners, replies back in the requesters' segment order
        replies = [[None] * W for _ in range(W)]
        for d in range(W):
            parts = [segs[r][d][:int(M[r, d])] for r in range(W)]
            rows_d = torch.cat(parts) if parts else None
            if rows_d is None or rows_d.shape[0] == 0:
                continue
            resp = steppers[d].serve(rows_d)
            off = 0
            for r in range(W):
                k = int(M[r, d])
                replies[r][d] = resp[off:off + k]
                off += k
        for r in range(W):
            parts = [x for x in replies[r] if x is not None and x.shape[0]]
            if parts:
                steppers[r].deliver(torch.cat(parts))
        if rounds > max_rounds:
            raise RuntimeError("sharded Kademlia routing did not terminate")
    return [s.finished() for s in steppers], rounds


def done_to_numpy(done_t) -> np.ndarray:
    return done_t.cpu().numpy().view(DONE_DTYPE).ravel()


def bench_exchange(device, comm_dev):
    """The native loop's exchange for a bench rank: the library's RCCL exchange when the process group
    is RCCL (comm_dev on the GPU), else torch.distributed callbacks (gloo rehearsal)."""
    if comm_dev is not None and getattr(comm_dev, "type", "cuda") == "cuda":
        return rccl_exchange_from_torch(device.index if device.index is not None else 0)
    return CallbackExchange(device).ex


class ShardedChord:
    """bench.py driver for one rank: ring arc + lookups resident in HBM + RCCL exchange.  The round loop
    runs in C++ behind the ABI (ovs_shard_route_batch) unless OVS_SHARD_PYLOOP=1 (the Python loop,
    route_sharded, over torch.distributed)."""

    def __init__(self, rank, world, ids, xy, keys_t, src_t, device, comm_dev=None, params=None, top_levels=None,
                 native=None):
        import os
        self.bounds = arc_bounds(len(ids), world)
        n = keys_t.shape[0]
        self.stepper = GpuShardStepper(ids, xy, self.bounds, rank, device, capacity=max(n + n // 4, 1024), params=params,
                                       top_levels=top_levels)
        self.stepper.reset(world * n + 1024)
        self.stepper.timing = True
        self.native = (os.environ.get("OVS_SHARD_PYLOOP") != "1") if native is None else native
        if self.native:
            self.ex = bench_exchange(device, comm_dev)
        else:
            self.exchange = TorchExchange(world, comm_dev if comm_dev is not None else device)
        self.keys_t, self.src_t = keys_t, src_t
        self.qid_base = rank * n
        self._done = None
        self.rounds = 0
        self.runs = 0
        self.kernel_ms = 0.0
        self.stats = None

    def run(self):
        self.stepper.reset(self.stepper.done_cap)
        self.stepper.kernel_ms = 0.0
        if self.native:
            self._done, st = native_route(self.stepper, self.ex, self.keys_t, self.src_t, self.qid_base, cohorts=2)
            self.rounds = st.rounds
            self.stats = st.as_dict()
            self.kernel_ms += st.step_ms
        else:
            self._done, self.rounds = route_sharded(self.stepper, self.exchange, self.keys_t, self.src_t, self.qid_base)
            self.kernel_ms += self.stepper.kernel_ms
        self.runs += 1

    def hop_total(self) -> int:
        d = done_to_numpy(self._done)
        return int(d["hops"].astype(np.int64).sum())

    def results_by_qid(self) -> dict:
        """This rank's finished records in batch order (qid - qid_base), as ovs_route_out fields."""
        return _results_by_qid(self._done, self.qid_base, self.keys_t.shape[0], rpcs=False)

    def ok_total(self) -> int:
        d = done_to_numpy(self._done)
        return int((d["status"] == 0).sum())


class ShardedKademlia:
    """bench.py driver for one rank: Kademlia arc + lookups resident in HBM + request/response exchange
    (the round loop in C++, ovs_kad_shard_route_batch, unless OVS_SHARD_PYLOOP=1)."""

    def __init__(self, rank, world, ids, xy, keys_t, src_t, device, comm_dev=None, params=None, native=None,
                 top_levels=None):
        import os
        self.bounds = arc_bounds(len(ids), world)
        # one-way routes on W > 1 arcs migrate over replicated top buckets (3 levels; the W = 8 E model:
        # 8.4 ms per arc against 32.8 ms with request/response rounds); OVS_KAD_TOP_LEVELS=0 keeps the
        # request/response rounds
        if top_levels is None:
            top_levels = int(os.environ.get("OVS_KAD_TOP_LEVELS", "3")) if world > 1 else 0
        self.stepper = KadShardStepper(ids, xy, self.bounds, rank, device, params=params, top_levels=top_levels)
        self.stepper.timing = True
        self.native = (os.environ.get("OVS_SHARD_PYLOOP") != "1") if native is None else native
        if self.native:
            self.ex = bench_exchange(device, comm_dev)
        else:
            self.exchange = TorchExchange(world, comm_dev if comm_dev is not None else device)
        self.stats = None
        self.keys_t, self.src_t = keys_t, src_t
        self.qid_base = rank * keys_t.shape[0]
        self._done = None
        self.rounds = 0
        self.runs = 0
        self.kernel_ms = 0.0
        self.served = 0

    def run(self):
        self.stepper.kernel_ms = 0.0
        self.stepper.served = 0
        if self.native:
            self._done, st = native_kad_route(self.stepper, self.ex, self.keys_t, self.src_t, self.qid_base)
            self.rounds = st.rounds
            self.stats = st.as_dict()
            self.kernel_ms += st.step_ms
        else:
            self._done, self.rounds = route_kad_sharded(self.stepper, self.exchange, self.keys_t, self.src_t,
                                                        self.qid_base)
            self.kernel_ms += self.stepper.kernel_ms
            self.served = self.stepper.served
        self.runs += 1

    def hop_total(self) -> int:
        return int(done_to_numpy(self._done)["hops"].astype(np.int64).sum())

    def ok_total(self) -> int:
        return int((done_to_numpy(self._done)["status"] == 0).sum())

    def rpc_total(self) -> int:
        """FindNodeCalls of this rank's lookups (the done records carry each lookup's count)."""
        return int(done_to_numpy(self._done)["pad"].astype(np.int64).sum())

    def results_by_qid(self) -> dict:
        """This rank's finished records in batch order, as ovs_route_out fields plus the RPC counts."""
        return _results_by_qid(self._done, self.qid_base, self.keys_t.shape[0], rpcs=True)


def _results_by_qid(done_t, qid_base: int, n: int, rpcs: bool) -> dict:
    d = done_to_numpy(done_t)
    i = d["qid"].astype(np.int64) - int(qid_base)
    if len(d) != n or i.min(initial=0) < 0 or i.max(initial=-1) >= n:
        raise RuntimeError(f"finished records do not cover the batch ({len(d)} for {n})")
    out = {}
    for f in ("responsible", "hops", "status", "one_way_hops", "latency_ns"):
        a = np.empty(n, dtype=d[f].dtype)
        a[i] = d[f]
        out[f] = a
    if rpcs:
        a = np.empty(n, dtype=np.uint32)
        a[i] = d["pad"]
        out["rpcs"] = a
    return out
