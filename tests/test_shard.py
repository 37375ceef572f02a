"""Multi-GPU (sharded ring) path.

CPU (world_size 2, gloo): route_sharded + TorchExchange + grouping/termination,
driven by a pure-Python stepper that restates the per-hop semantics (refmodel).
GPU: the ovs_shard_step kernel with W arcs emulated in one process, and two
processes sharing cuda:0 with a gloo exchange; both compared with the
single-GPU engine and the oracle.
"""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch

import refmodel
from oversim_amd import workload as W

ROUTE_FIELDS = ("responsible", "hops", "status", "one_way_hops", "latency_ns")


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class CpuShardStepper:
    """Test double of GpuShardStepper: same record format, per-hop logic from refmodel."""

    def __init__(self, ids, xy, bounds, rank):
        from oversim_amd.shard import DONE_DTYPE, REC_DTYPE
        self.REC, self.DONE = REC_DTYPE, DONE_DTYPE
        self.ring = refmodel.ChordRing(ids, xy)
        self.lo, self.hi = bounds[rank], bounds[rank + 1]
        self.bounds = bounds
        self.done = []
        self.dev = torch.device("cpu")

    def make_records(self, keys_t, src_t, qid_base):
        keys, src = keys_t.numpy(), src_t.numpy()
        r = np.zeros(len(keys), dtype=self.REC)
        r["key"], r["src"], r["cur"] = keys, src, src
        r["qid"] = qid_base + np.arange(len(keys))
        r["local"] = 1
        return torch.from_numpy(r.view(np.uint8).reshape(-1, 48).copy())

    def owner(self, c):
        return int(np.searchsorted(self.bounds, c, side="right") - 1)

    def cohort(self, c):
        from oversim_amd.shard import _NoCtx
        return _NoCtx()

    def step(self, inbox, cohort=0):
        recs = inbox.numpy().view(self.REC).ravel()
        out, dest = [], []
        ring = self.ring
        call, resp, route = refmodel.msg_ns(83), refmodel.msg_ns(87), refmodel.msg_ns(186)
        for rec in recs:
            K = refmodel.to_int(rec["key"])
            S, cur, t, hops, local = int(rec["src"]), int(rec["cur"]), int(rec["t_ns"]), int(rec["hops"]), bool(rec["local"])
            while True:
                assert self.lo <= cur < self.hi
                sib, nxt = ring.decide(cur, K)
                status, R = None, None
                if local:
                    local = False
                    if sib:
                        status, R = 0, S
                else:
                    cd = refmodel.coord_ns(ring.xy, S, cur)
                    t += call + resp + 2 * cd
                    hops += 1
                    if sib:
                        status, R = 0, cur
                if status is None:
                    if hops >= 50:
                        status = 3
                    elif nxt == S:
                        status = 4
                if status is not None:
                    lat = t + (route + refmodel.coord_ns(ring.xy, S, R) if (status == 0 and R != S) else 0)
                    self.done.append((int(rec["qid"]), R if status == 0 else 0xFFFFFFFF, hops, status,
                                      hops + (R != S) if status == 0 else 0, lat if status == 0 else -1))
                    break
                cur = nxt
                if not (self.lo <= cur < self.hi):
                    o = rec.copy()
                    o["cur"], o["t_ns"], o["hops"], o["local"] = cur, t, hops, 0
                    out.append(o)
                    dest.append(self.owner(cur))
                    break
        # per-destination send segments, as the kernel writes them
        world = len(self.bounds) - 1
        segs = []
        for d in range(world):
            o = [r for r, x in zip(out, dest) if x == d]
            o = np.array(o, dtype=self.REC) if o else np.zeros(0, dtype=self.REC)
            segs.append(torch.from_numpy(o.view(np.uint8).reshape(-1, 48).copy()))
        return segs, torch.tensor([s.shape[0] for s in segs], dtype=torch.int64)

    def finished(self):
        d = np.zeros(len(self.done), dtype=self.DONE)
        for i, (q, R, h, st, ow, lat) in enumerate(self.done):
            d[i]["qid"], d[i]["responsible"], d[i]["hops"], d[i]["status"] = q, R, h, st
            d[i]["one_way_hops"], d[i]["latency_ns"] = ow, lat
        return torch.from_numpy(d.view(np.uint8).reshape(-1, 24).copy())


def _cpu_worker(rank, world, port, n, m, q, cohorts=1):
    import torch.distributed as dist
    from oversim_amd.shard import TorchExchange, arc_bounds, done_to_numpy, route_sharded
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    net = W.population(n, 91)
    bounds = arc_bounds(n, world)
    keys, src = W.lookups(net.ids, m, 92 + rank, node_ids=rank == 0)
    src = (bounds[rank] + src.astype(np.int64) % (bounds[rank + 1] - bounds[rank])).astype(np.uint32)
    st = CpuShardStepper(net.ids, net.xy, bounds, rank)
    done, rounds = route_sharded(st, TorchExchange(world, torch.device("cpu")), torch.from_numpy(keys),
                                 torch.from_numpy(src), rank * m, cohorts=cohorts, min_split=1)
    q.put((rank, done_to_numpy(done), keys, src, rounds))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,cohorts", [(2, 1), (2, 2), (3, 3)])
def test_sharded_orchestration_gloo_cpu(world, cohorts):
    """cohorts > 1: the lookups of a rank in cohorts whose exchanges interleave (route_sharded)."""
    import torch.multiprocessing as mp
    n, m = 600, 300
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_cpu_worker, args=(r, world, port, n, m, q, cohorts)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    net = W.population(n, 91)
    ring = refmodel.ChordRing(net.ids, net.xy)
    all_done = np.concatenate([r[1] for r in res])
    assert len(all_done) == world * m and len(np.unique(all_done["qid"])) == world * m
    by_q = {int(d["qid"]): d for d in all_done}
    for rank, _, keys, src, rounds in res:
        assert rounds >= 2
        for i in range(m):
            ref = ring.lookup(keys[i], int(src[i]))
            d = by_q[rank * m + i]
            for f in ROUTE_FIELDS:
                assert int(d[f]) == int(ref[f]), (rank, i, f)


# ---------------------------------------------------------------------------- GPU

def _single_gpu_reference(net, keys, src, routing_type=0):
    from oversim_amd import KbrEngine, Params
    with KbrEngine(0) as e:
        e.set_params(Params.chord().replace(routingType=routing_type))
        e.chord_load(net.ids, net.xy)
        return e.lookup(keys, src)


@pytest.mark.gpu
@pytest.mark.parametrize("world,rt,ext,top,n", [
    (2, 0, 0, None, 1 << 16), (3, 0, 0, None, 1 << 16), (8, 0, 0, None, 1 << 16), (3, 1, 0, None, 1 << 16),
    (8, 1, 0, None, 1 << 16), (3, 0, 1, None, 1 << 16),
    # no replicated levels (every off-arc responder handed to its owner)
    (3, 0, 0, 0, 1 << 16), (8, 1, 0, 0, 1 << 16),
    # small rings with many replicated levels: off-arc responders that need their successor window or a
    # finger below the replicated levels go to their owner as "reached" records (local byte 2)
    (8, 0, 0, 32, 600), (3, 1, 0, 32, 300), (4, 0, 0, 12, 5000), (2, 0, 1, 20, 1 << 16), (2, 0, 0, 20, 2000)])
def test_shard_step_emulated_on_one_gpu(world, rt, ext, top, n):
    """rt = routingType: 0 iterative, 1 semi-recursive (ChordLarge).  ext: the arcs route with
    extendedFingerTable = true (no call can time out on this field: equal to the plain table).
    top: replicated top finger levels (ovs_chord_shard_replicate; None = the default for the world)."""
    from oversim_amd import Params
    from oversim_amd.shard import GpuShardStepper, arc_bounds, done_to_numpy, route_local_shards
    m = 6000
    net = W.population(n, 93)
    bounds = arc_bounds(n, world)
    dev = torch.device("cuda", 0)
    params = Params.chord().replace(routingType=rt, extendedFingerTable=ext)
    steppers = [GpuShardStepper(net.ids, net.xy, bounds, r, dev, capacity=world * m, params=params, top_levels=top)
                for r in range(world)]
    ks, ss, qb, allk, alls = [], [], [], [], []
    for r in range(world):
        k, s = W.lookups(net.ids, m, 94 + r, node_ids=(r % 2 == 0))
        s = (bounds[r] + s.astype(np.int64) % (bounds[r + 1] - bounds[r])).astype(np.uint32)
        ks.append(torch.from_numpy(k).to(dev)); ss.append(torch.from_numpy(s).to(dev)); qb.append(r * m)
        allk.append(k); alls.append(s)
    for st in steppers:
        st.reset(world * m)
    dones, rounds = route_local_shards(steppers, ks, ss, qb)
    d = np.concatenate([done_to_numpy(x) for x in dones])
    d = d[np.argsort(d["qid"])]
    assert np.array_equal(d["qid"], np.arange(world * m))
    ref = _single_gpu_reference(net, np.concatenate(allk), np.concatenate(alls), rt)
    for f in ROUTE_FIELDS:
        assert np.array_equal(d[f].astype(np.int64), ref[f].astype(np.int64)), f
    assert rounds >= 2


def _gpu_worker(rank, world, port, q):
    import torch.distributed as dist
    from oversim_amd.shard import GpuShardStepper, TorchExchange, arc_bounds, done_to_numpy, route_sharded
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n, m = 1 << 15, 4000
    net = W.population(n, 95)
    bounds = arc_bounds(n, world)
    k, s = W.lookups(net.ids, m, 96 + rank, node_ids=False)
    s = (bounds[rank] + s.astype(np.int64) % (bounds[rank + 1] - bounds[rank])).astype(np.uint32)
    dev = torch.device("cuda", 0)
    st = GpuShardStepper(net.ids, net.xy, bounds, rank, dev, capacity=world * m)
    st.reset(world * m)
    # two cohorts on two HIP streams (the exchange of one overlaps the kernel of the other)
    done, rounds = route_sharded(st, TorchExchange(world, torch.device("cpu")), torch.from_numpy(k).to(dev),
                                 torch.from_numpy(s).to(dev), rank * m, cohorts=2, min_split=1)
    q.put((rank, done_to_numpy(done), k, s))
    dist.barrier()
    dist.destroy_process_group()


class _SelfExchange:
    """world = 1 exchange (no process group): every record stays on rank 0."""
    rank, world = 0, 1

    def count_matrix_async(self, counts):
        M = counts.reshape(1, -1).cpu().numpy()
        return lambda: M

    def segments(self, segs, scl, rcl, row_bytes):
        return segs[0][:rcl[0]].clone()


@pytest.mark.gpu
@pytest.mark.parametrize("cohorts", [2, 3])
def test_cohorts_share_the_done_buffer(cohorts):
    """Cohorts on their own streams append to one done buffer: the compaction reserves each cohort's
    records with an atomic (a plain read-modify-write of the shared counter let two cohorts take the
    same positions).  Uneven cohorts, repeated batches: every qid exactly once, equal to
    the single-GPU route."""
    from oversim_amd.shard import GpuShardStepper, arc_bounds, done_to_numpy, route_sharded
    n, m = 1 << 15, 10_007
    net = W.population(n, 95)
    k, s = W.lookups(net.ids, m, 77, node_ids=False)
    dev = torch.device("cuda", 0)
    st = GpuShardStepper(net.ids, net.xy, arc_bounds(n, 1), 0, dev, capacity=m)
    ref = _single_gpu_reference(net, k, s)
    kt, sv = torch.from_numpy(k).to(dev), torch.from_numpy(s).to(dev)
    for rep in range(6):
        st.reset(m)
        done, _ = route_sharded(st, _SelfExchange(), kt, sv, 0, cohorts=cohorts, min_split=1)
        d = done_to_numpy(done)
        assert len(d) == m, (rep, len(d))
        d = d[np.argsort(d["qid"])]
        assert np.array_equal(d["qid"], np.arange(m)), rep
        for f in ROUTE_FIELDS:
            assert np.array_equal(d[f].astype(np.int64), ref[f].astype(np.int64)), (rep, f)


@pytest.mark.gpu
def test_two_processes_share_one_gpu_gloo():
    import torch.multiprocessing as mp
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gpu_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=600) for _ in range(world)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    d = np.concatenate([r[1] for r in res])
    d = d[np.argsort(d["qid"])]
    net = W.population(1 << 15, 95)
    ref = _single_gpu_reference(net, np.concatenate([r[2] for r in res]), np.concatenate([r[3] for r in res]))
    for f in ROUTE_FIELDS:
        assert np.array_equal(d[f].astype(np.int64), ref[f].astype(np.int64)), f


# ------------------------------------------------------------- Kademlia request/response

class FakeKadStepper:
    """Protocol double for route_kad_sharded: lookup i queries the nodes plan[i] one after the
    other; each query is a request to the node's owner, answered with a value derived from
    (node, key) that the requester checks.  Exercises the per-owner segments, the count matrix,
    both all-to-allv directions (reverse splits), delivery by tag and termination -- without a GPU."""

    def __init__(self, bounds, rank, n_nodes, seed):
        self.bounds, self.rank, self.world = bounds, rank, len(bounds) - 1
        self.dev = torch.device("cpu")
        self.rng = np.random.default_rng(seed)
        self.n_nodes = n_nodes
        self.served = 0

    def owner(self, c):
        return int(np.searchsorted(self.bounds, c, side="right") - 1)

    def begin(self, keys_t, src_t, qid_base):
        n = keys_t.shape[0]
        self.keys = keys_t.numpy()
        self.plan = [list(self.rng.integers(0, self.n_nodes, int(self.rng.integers(1, 6)))) for _ in range(n)]
        self.pos = [0] * n
        self.waiting = [False] * n
        self.acc = [0] * n
        self.qid_base = qid_base
        self.done = []

    def step(self):
        segs = [[] for _ in range(self.world)]
        active = 0
        for i in range(len(self.plan)):
            if self.waiting[i] or self.pos[i] < 0:
                if self.waiting[i]:
                    active += 1
                continue
            if self.pos[i] == len(self.plan[i]):
                self.done.append((self.qid_base + i, self.acc[i]))
                self.pos[i] = -1
                continue
            node = int(self.plan[i][self.pos[i]])
            rec = np.zeros(8, np.uint32)
            rec[:5] = self.keys[i]
            rec[5], rec[6] = node, i
            segs[self.owner(node)].append(rec.view(np.uint8))
            self.waiting[i] = True
            active += 1
        out = [torch.from_numpy(np.stack(x)) if x else torch.zeros((0, 32), dtype=torch.uint8) for x in segs]
        counts = torch.tensor([x.shape[0] for x in out] + [active, len(self.done)], dtype=torch.int64)
        return out, counts

    def serve(self, reqs):
        r = reqs.numpy().view(np.uint32).reshape(-1, 8)
        resp = np.zeros((len(r), 26), np.uint32)
        for j, q in enumerate(r):
            assert self.bounds[self.rank] <= q[5] < self.bounds[self.rank + 1], "request at the wrong owner"
            resp[j, 0] = q[6]
            resp[j, 1] = (int(q[5]) * 2654435761 + int(q[0])) & 0xFFFFFFFF
        self.served += len(r)
        return torch.from_numpy(resp.view(np.uint8).reshape(-1, 104).copy())

    def deliver(self, resps):
        r = resps.numpy().view(np.uint32).reshape(-1, 26)
        for q in r:
            i = int(q[0])
            node = int(self.plan[i][self.pos[i]])
            assert q[1] == (node * 2654435761 + int(self.keys[i][0])) & 0xFFFFFFFF, "response for another query"
            self.acc[i] = (self.acc[i] * 31 + int(q[1])) & 0xFFFFFFFF
            self.pos[i] += 1
            self.waiting[i] = False

    def finished(self):
        return self.done


def _expected_acc(keys, plan):
    acc = 0
    for node in plan:
        acc = (acc * 31 + ((int(node) * 2654435761 + int(keys[0])) & 0xFFFFFFFF)) & 0xFFFFFFFF
    return acc


def _kad_cpu_worker(rank, world, port, q):
    import torch.distributed as dist
    from oversim_amd.shard import TorchExchange, arc_bounds, route_kad_sharded
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n_nodes, m = 1000, 200
    bounds = arc_bounds(n_nodes, world)
    keys = W.random_keys(m, np.random.default_rng(50 + rank))
    st = FakeKadStepper(bounds, rank, n_nodes, 60 + rank)
    done, rounds = route_kad_sharded(st, TorchExchange(world, torch.device("cpu")), torch.from_numpy(keys),
                                     torch.zeros(m, dtype=torch.int32), rank * m)
    q.put((rank, done, [list(map(int, p)) for p in st.plan], keys, rounds, st.served))
    dist.barrier()
    dist.destroy_process_group()


def test_kad_request_response_orchestration_gloo_cpu():
    import torch.multiprocessing as mp
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_kad_cpu_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    total_q = sum(len(pl) for r in res for pl in r[2])
    assert sum(r[5] for r in res) == total_q                  # every query served exactly once
    longest = max(len(pl) for r in res for pl in r[2])
    for rank, done, plan, keys, rounds, _ in res:
        assert rounds == longest + 1                          # one round per query + the finishing step
        got = dict(done)
        assert len(got) == len(plan)
        for i, p in enumerate(plan):
            assert got[rank * len(plan) + i] == _expected_acc(keys[i], p)


def _kad_reference(net, keys, src, params):
    from oversim_amd import KbrEngine
    with KbrEngine(0) as e:
        e.set_params(params)
        e.kad_load(net.ids, net.xy)
        return e.lookup(keys, src, count_rpcs=True)


@pytest.mark.gpu
@pytest.mark.parametrize("world,alpha,n", [(2, 1, 15000), (3, 3, 15000), (8, 3, 1 << 16), (4, 2, 1 << 16), (3, 8, 15000),
                                           (2, 5, 15000)])
def test_kad_shards_emulated_on_one_gpu(world, alpha, n):
    """W arcs in one process: every lookup's result equals the single-GPU kernel's."""
    from oversim_amd import Params
    from oversim_amd.shard import KadShardStepper, arc_bounds, done_to_numpy, route_kad_local_shards
    m = 4000
    net = W.population(n, 97)
    bounds = arc_bounds(n, world)
    dev = torch.device("cuda", 0)
    params = Params.kademlia().replace(lookupParallelRpcs=alpha)
    steppers = [KadShardStepper(net.ids, net.xy, bounds, r, dev, params=params) for r in range(world)]
    ks, ss, qb, allk, alls = [], [], [], [], []
    for r in range(world):
        k, s = W.lookups(net.ids, m, 98 + r, node_ids=(r % 2 == 0))
        s = (bounds[r] + s.astype(np.int64) % (bounds[r + 1] - bounds[r])).astype(np.uint32)
        ks.append(torch.from_numpy(k.view(np.int32)).to(dev))
        ss.append(torch.from_numpy(s.view(np.int32)).to(dev))
        qb.append(r * m)
        allk.append(k); alls.append(s)
    dones, rounds = route_kad_local_shards(steppers, ks, ss, qb)
    d = np.concatenate([done_to_numpy(x) for x in dones])
    d = d[np.argsort(d["qid"])]
    assert np.array_equal(d["qid"], np.arange(world * m))
    ref = _kad_reference(net, np.concatenate(allk), np.concatenate(alls), params)
    for f in ROUTE_FIELDS:
        assert np.array_equal(d[f].astype(np.int64), ref[f].astype(np.int64)), f
    assert np.array_equal(d["pad"].astype(np.int64), ref["rpcs"].astype(np.int64))   # FindNodeCalls per lookup
    assert rounds >= 3


def _kad_gpu_worker(rank, world, port, q, ns=None):
    import torch.distributed as dist
    from oversim_amd import Params
    from oversim_amd.shard import KadShardStepper, TorchExchange, arc_bounds, done_to_numpy, route_kad_sharded
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n, m = 1 << 15, 3000
    net = W.population(n, 99)
    bounds = arc_bounds(n, world)
    k, s = W.lookups(net.ids, m, 100 + rank, node_ids=ns is not None)
    s = (bounds[rank] + s.astype(np.int64) % (bounds[rank + 1] - bounds[rank])).astype(np.uint32)
    dev = torch.device("cuda", 0)
    st = KadShardStepper(net.ids, net.xy, bounds, rank, dev, params=Params.kademlia(), lookup_siblings=ns)
    done, rounds = route_kad_sharded(st, TorchExchange(world, torch.device("cpu")),
                                     torch.from_numpy(k.view(np.int32)).to(dev),
                                     torch.from_numpy(s.view(np.int32)).to(dev), rank * m)
    if ns is None:
        q.put((rank, done_to_numpy(done), k, s))
    else:
        q.put((rank, st.lookup_results(done), k, s))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
def test_kad_lookup_calls_two_processes_share_one_gpu_gloo():
    """Sharded Kademlia LookupCalls (numSiblings = s) with the request/response exchange between two
    processes: every LookupResponse equals the single-context ovs_lookup_batch's."""
    import torch.multiprocessing as mp
    from oversim_amd import KbrEngine, Params
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_kad_gpu_worker, args=(r, world, port, q, -1)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=600) for _ in range(world)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    qid = np.concatenate([r[1][0] for r in res])
    lo = np.concatenate([r[1][1] for r in res])
    sib = np.concatenate([r[1][2] for r in res])
    order = np.argsort(qid)
    assert np.array_equal(qid[order], np.arange(world * 3000))
    lo, sib = lo[order], sib[order]
    net = W.population(1 << 15, 99)
    with KbrEngine(0) as eng:
        eng.set_params(Params.kademlia())
        eng.kad_load(net.ids, net.xy)
        ref = eng.lookupCall(np.concatenate([r[2] for r in res]), np.concatenate([r[3] for r in res]), -1)
    for f in ("num_siblings", "hops", "status", "is_valid", "latency_ns"):
        assert np.array_equal(lo[f], ref[f]), f
    assert np.array_equal(sib, ref["siblings"])
    assert lo["is_valid"].mean() > 0.99


@pytest.mark.gpu
def test_kad_two_processes_share_one_gpu_gloo():
    import torch.multiprocessing as mp
    from oversim_amd import Params
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_kad_gpu_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=600) for _ in range(world)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    d = np.concatenate([r[1] for r in res])
    d = d[np.argsort(d["qid"])]
    net = W.population(1 << 15, 99)
    ref = _kad_reference(net, np.concatenate([r[2] for r in res]), np.concatenate([r[3] for r in res]),
                         Params.kademlia())
    for f in ROUTE_FIELDS:
        assert np.array_equal(d[f].astype(np.int64), ref[f].astype(np.int64)), f


# ------------------------------------------------------------- W = 8 at 2^22 nodes vs the oracle

@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_chord_w8_large_ring_vs_oracle():
    """Eight arcs of a 2^22-node ring (one context per arc on one GPU, the in-process exchange):
    every lookup compared with the CPU oracle itself, not with the single-GPU kernel."""
    from oversim_amd import Params
    from oversim_amd.shard import GpuShardStepper, arc_bounds, done_to_numpy, route_local_shards
    from oracle_lib import OracleNet
    world, n, m = 8, 1 << 22, 12_500
    net = W.population(n, 191)
    bounds = arc_bounds(n, world)
    dev = torch.device("cuda", 0)
    steppers = [GpuShardStepper(net.ids, net.xy, bounds, r, dev, capacity=world * m, params=Params.chord())
                for r in range(world)]
    ks, ss, qb, allk, alls = [], [], [], [], []
    for r in range(world):
        k, s = W.lookups(net.ids, m, 192 + r, node_ids=(r % 2 == 0))
        s = (bounds[r] + s.astype(np.int64) % (bounds[r + 1] - bounds[r])).astype(np.uint32)
        ks.append(torch.from_numpy(k).to(dev)); ss.append(torch.from_numpy(s).to(dev)); qb.append(r * m)
        allk.append(k); alls.append(s)
    for st in steppers:
        st.reset(world * m)
    dones, rounds = route_local_shards(steppers, ks, ss, qb)
    d = np.concatenate([done_to_numpy(x) for x in dones])
    d = d[np.argsort(d["qid"])]
    assert np.array_equal(d["qid"], np.arange(world * m))
    ref = OracleNet("chord", net.ids, net.xy, lazy=True).route(np.concatenate(allk), np.concatenate(alls),
                                                               record_hops=False)
    for f in ROUTE_FIELDS:
        assert np.array_equal(d[f].astype(np.int64), ref[f].astype(np.int64)), f
    # with the replicated top levels a lookup crosses arcs about once: 2-3 rounds (5 without)
    assert rounds >= 2


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_kad_w8_large_network_vs_oracle():
    """Eight ID arcs of a 2^22-node Kademlia network, alpha = 3, request/response exchange in one
    process: every lookup (and its RPC count) compared with the CPU oracle."""
    from oversim_amd import Params
    from oversim_amd.shard import KadShardStepper, arc_bounds, done_to_numpy, route_kad_local_shards
    from oracle_lib import OracleNet, kad_params
    world, n, m = 8, 1 << 22, 5_000
    net = W.population(n, 193)
    bounds = arc_bounds(n, world)
    dev = torch.device("cuda", 0)
    params = Params.kademlia().replace(lookupParallelRpcs=3)
    steppers = [KadShardStepper(net.ids, net.xy, bounds, r, dev, params=params) for r in range(world)]
    ks, ss, qb, allk, alls = [], [], [], [], []
    for r in range(world):
        k, s = W.lookups(net.ids, m, 194 + r, node_ids=(r % 2 == 1))
        s = (bounds[r] + s.astype(np.int64) % (bounds[r + 1] - bounds[r])).astype(np.uint32)
        ks.append(torch.from_numpy(k.view(np.int32)).to(dev))
        ss.append(torch.from_numpy(s.view(np.int32)).to(dev))
        qb.append(r * m)
        allk.append(k); alls.append(s)
    dones, rounds = route_kad_local_shards(steppers, ks, ss, qb)
    d = np.concatenate([done_to_numpy(x) for x in dones])
    d = d[np.argsort(d["qid"])]
    assert np.array_equal(d["qid"], np.arange(world * m))
    ref = OracleNet("kademlia", net.ids, net.xy, kad_params(lookupParallelRpcs=3), lazy=True).route(
        np.concatenate(allk), np.concatenate(alls), record_hops=False)
    for f in ROUTE_FIELDS:
        assert np.array_equal(d[f].astype(np.int64), ref[f].astype(np.int64)), f
    assert sum(s.served for s in steppers) > world * m


@pytest.mark.gpu
@pytest.mark.parametrize("world,ns", [(2, 8), (3, 5), (8, 8)])
def test_shard_lookup_calls_emulated_on_one_gpu(world, ns):
    """KBRTestApp LookupCalls across W arcs (ovs_shard_step_lookup + ovs_shard_lookup_finish): every
    LookupResponse equals the single-context ovs_lookup_batch's (itself checked against the oracle)."""
    from oversim_amd import KbrEngine, Params
    from oversim_amd.shard import GpuShardStepper, arc_bounds, route_local_shards
    n, m = 1 << 16, 5000
    net = W.population(n, 97)
    bounds = arc_bounds(n, world)
    dev = torch.device("cuda", 0)
    steppers = [GpuShardStepper(net.ids, net.xy, bounds, r, dev, capacity=world * m, lookup_siblings=ns)
                for r in range(world)]
    ks, ss, qb, allk, alls = [], [], [], [], []
    for r in range(world):
        k, s = W.lookups(net.ids, m, 98 + r, node_ids=(r % 2 == 1))
        s = (bounds[r] + s.astype(np.int64) % (bounds[r + 1] - bounds[r])).astype(np.uint32)
        ks.append(torch.from_numpy(k).to(dev)); ss.append(torch.from_numpy(s).to(dev)); qb.append(r * m)
        allk.append(k); alls.append(s)
    for st in steppers:
        st.reset(world * m)
    dones, rounds = route_local_shards(steppers, ks, ss, qb)
    parts = [steppers[r].lookup_finish(dones[r]) for r in range(world)]
    qid = np.concatenate([p[0] for p in parts])
    lo = np.concatenate([p[1] for p in parts])
    sib = np.concatenate([p[2] for p in parts])
    order = np.argsort(qid)
    assert np.array_equal(qid[order], np.arange(world * m))
    lo, sib = lo[order], sib[order]
    with KbrEngine(0) as eng:
        eng.set_params(Params.chord())
        eng.chord_load(net.ids, net.xy)
        ref = eng.lookupCall(np.concatenate(allk), np.concatenate(alls), ns)
    for f in ("num_siblings", "hops", "status", "is_valid", "latency_ns"):
        assert np.array_equal(lo[f], ref[f]), f
    assert np.array_equal(sib, ref["siblings"])
    assert rounds >= 2


@pytest.mark.gpu
@pytest.mark.parametrize("world,alpha,ns", [(2, 3, 8), (3, 1, 3), (4, 3, 0), (8, 2, -1)])
def test_kad_shard_lookup_calls_emulated_on_one_gpu(world, alpha, ns):
    """KBRTestApp LookupCalls on W Kademlia arcs (ovs_kad_shard_begin_lookup): the requests carry
    numSiblings to the serving rank; every LookupResponse and sibling row equals the single-context
    ovs_lookup_batch's (itself checked against the oracle in test_gpu_lookupcall.py).  ns = 0 is
    the exact-key lookup."""
    from oversim_amd import KbrEngine, Params
    from oversim_amd.shard import KadShardStepper, arc_bounds, route_kad_local_shards
    n, m = 1 << 15, 3000
    net = W.population(n, 97)
    bounds = arc_bounds(n, world)
    dev = torch.device("cuda", 0)
    params = Params.kademlia().replace(lookupParallelRpcs=alpha)
    steppers = [KadShardStepper(net.ids, net.xy, bounds, r, dev, params=params, lookup_siblings=ns)
                for r in range(world)]
    ks, ss, qb, allk, alls = [], [], [], [], []
    for r in range(world):
        k, s = W.lookups(net.ids, m, 98 + r, node_ids=(ns == 0 or r % 2 == 1))
        s = (bounds[r] + s.astype(np.int64) % (bounds[r + 1] - bounds[r])).astype(np.uint32)
        ks.append(torch.from_numpy(k.view(np.int32)).to(dev))
        ss.append(torch.from_numpy(s.view(np.int32)).to(dev))
        qb.append(r * m)
        allk.append(k); alls.append(s)
    dones, rounds = route_kad_local_shards(steppers, ks, ss, qb)
    parts = [steppers[r].lookup_results(dones[r]) for r in range(world)]
    qid = np.concatenate([p[0] for p in parts])
    lo = np.concatenate([p[1] for p in parts])
    sib = np.concatenate([p[2] for p in parts])
    order = np.argsort(qid)
    assert np.array_equal(qid[order], np.arange(world * m))
    lo, sib = lo[order], sib[order]
    with KbrEngine(0) as eng:
        eng.set_params(params)
        eng.kad_load(net.ids, net.xy)
        ref = eng.lookupCall(np.concatenate(allk), np.concatenate(alls), ns)
    for f in ("num_siblings", "hops", "status", "is_valid", "latency_ns"):
        assert np.array_equal(lo[f], ref[f]), f
    assert np.array_equal(sib, ref["siblings"])
    assert (lo["is_valid"] == 1).mean() > 0.9
    assert rounds >= 3


@pytest.mark.gpu
def test_kad_shard_source_off_arc_is_an_error():
    """A lookup whose source lies on another rank's arc never runs and is reported by
    ovs_kad_shard_errors (its own findNode needs that rank's rows)."""
    from oversim_amd.shard import KadShardStepper, arc_bounds, route_kad_local_shards
    n, world = 1 << 14, 2
    net = W.population(n, 97)
    bounds = arc_bounds(n, world)
    dev = torch.device("cuda", 0)
    steppers = [KadShardStepper(net.ids, net.xy, bounds, r, dev) for r in range(world)]
    k, _ = W.lookups(net.ids, 4, 5, node_ids=False)
    s_ok = np.full(4, bounds[0], dtype=np.uint32)
    s_bad = s_ok.copy()
    s_bad[2] = bounds[1]            # on arc 1, handed to rank 0
    kt = torch.from_numpy(k.view(np.int32)).to(dev)
    with pytest.raises(RuntimeError, match="could not be delivered"):
        route_kad_local_shards(steppers, [kt, kt], [torch.from_numpy(s_bad.view(np.int32)).to(dev),
                                                    torch.from_numpy((s_ok + bounds[1]).view(np.int32)).to(dev)],
                               [0, 4])


@pytest.mark.gpu
def test_kad_serve_refuses_requests_it_cannot_answer():
    """k_kad_shard_serve answers a request for a node off its arc, or with a numSiblings the home rank
    would have refused (> min(8, 5s)), as undeliverable (count 0xFFFFFFFF) instead of reading tables it
    does not hold; the requester's deliver counts it (ovs_kad_shard_errors)."""
    from oversim_amd.shard import KAD_REQ_DTYPE, KAD_RESP_DTYPE, KadShardStepper, arc_bounds
    n, world = 1 << 14, 2
    net = W.population(n, 97)
    bounds = arc_bounds(n, world)
    dev = torch.device("cuda", 0)
    st = KadShardStepper(net.ids, net.xy, bounds, 0, dev, lookup_siblings=8)
    k, _ = W.lookups(net.ids, 3, 5, node_ids=False)
    q = np.zeros(3, dtype=KAD_REQ_DTYPE)
    q["key"] = k
    q["node"] = [5, bounds[1] + 7, 9]                  # on the arc, off the arc, on the arc
    q["tag"] = [0, 1, 2]
    q["pad"] = [0x80000000 | 8, 0x80000000 | 8, 0x80000000 | 200]
    resp = st.serve(torch.from_numpy(q.view(np.uint8).reshape(3, -1).copy()).to(dev))
    r = resp.cpu().numpy().view(KAD_RESP_DTYPE).ravel()
    assert r["count"][0] <= 8 and r["count"][1] == 0xFFFFFFFF and r["count"][2] == 0xFFFFFFFF


def test_check_complete_reports_unwritten_rows_and_missing_records():
    """A finished record read from an exchange row nobody wrote (the 0xFF sentinel) or a record count
    that does not match the batch raises, instead of passing as lost lookups."""
    import torch
    from oversim_amd.shard import DONE_BYTES, check_complete
    ok = torch.zeros((5, DONE_BYTES), dtype=torch.uint8)
    check_complete(ok, 5, "t")
    bad = ok.clone()
    bad[2] = 0xFF
    with pytest.raises(RuntimeError, match="unwritten"):
        check_complete(bad, 5, "t")
    with pytest.raises(RuntimeError, match="4 finished records for 5"):
        check_complete(ok[:4], 5, "t")


# ------------------------------------------------- the round loop behind the C ABI (ABI 11)

def _native_inputs(net, bounds, world, m, seed, node_ids=lambda r: r % 2 == 0):
    ks, ss, allk, alls = [], [], [], []
    dev = torch.device("cuda", 0)
    for r in range(world):
        k, s = W.lookups(net.ids, m, seed + r, node_ids=node_ids(r))
        s = (bounds[r] + s.astype(np.int64) % (bounds[r + 1] - bounds[r])).astype(np.uint32)
        ks.append(torch.from_numpy(k.view(np.int32)).to(dev))
        ss.append(torch.from_numpy(s.view(np.int32)).to(dev))
        allk.append(k); alls.append(s)
    return ks, ss, np.concatenate(allk), np.concatenate(alls)


@pytest.mark.gpu
@pytest.mark.parametrize("kind,world,top", [("chord", 3, None), ("chord", 4, 0), ("chord", 2, 8), ("kademlia", 3, 0),
                                            ("kademlia", 3, 3), ("kademlia", 8, 2)])
def test_native_round_loop_threads(kind, world, top):
    """ovs_shard_route_batch / ovs_kad_shard_route_batch with W ranks as threads of this process (one
    context per arc on one GPU, ovs_exchange_local_create): equal to the single-context route."""
    import threading
    from oversim_amd import Params
    from oversim_amd.shard import (GpuShardStepper, KadShardStepper, arc_bounds, done_to_numpy, local_exchanges,
                                   native_kad_route, native_route, destroy_exchange)
    n, m = 1 << 15, 5000
    net = W.population(n, 0x5A + world)
    bounds = arc_bounds(n, world)
    dev = torch.device("cuda", 0)
    ks, ss, allk, alls = _native_inputs(net, bounds, world, m, 0x5B)
    if kind == "chord":
        steppers = [GpuShardStepper(net.ids, net.xy, bounds, r, dev, capacity=m, top_levels=top) for r in range(world)]
        for st in steppers:
            st.reset(world * m)
    else:
        params = Params.kademlia().replace(lookupParallelRpcs=3)
        # top > 0: replicated top buckets, the lookups migrate (ovs_kad_shard_mig_step rounds)
        steppers = [KadShardStepper(net.ids, net.xy, bounds, r, dev, params=params, top_levels=top or 0)
                    for r in range(world)]
    exs = local_exchanges(world)
    res, errs = [None] * world, []

    def run(r):
        try:
            with torch.cuda.device(dev):
                if kind == "chord":
                    res[r] = native_route(steppers[r], exs[r], ks[r], ss[r], r * m, cohorts=2)
                else:
                    res[r] = native_kad_route(steppers[r], exs[r], ks[r], ss[r], r * m)
        except Exception as e:       # noqa: BLE001
            errs.append(e)

    th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not errs, errs
    for ex in exs:
        destroy_exchange(ex)
    d = np.concatenate([done_to_numpy(x[0]) for x in res])
    d = d[np.argsort(d["qid"])]
    assert np.array_equal(d["qid"], np.arange(world * m))
    assert all(x[1].rounds >= 2 for x in res)
    if kind == "chord":
        ref = _single_gpu_reference(net, allk, alls)
    else:
        ref = _kad_reference(net, allk, alls, Params.kademlia().replace(lookupParallelRpcs=3))
        assert np.array_equal(d["pad"].astype(np.int64), ref["rpcs"].astype(np.int64))
    for f in ROUTE_FIELDS:
        assert np.array_equal(d[f].astype(np.int64), ref[f].astype(np.int64)), f


@pytest.mark.gpu
@pytest.mark.parametrize("kind,top", [("chord", None), ("kademlia", 0), ("kademlia", 3)])
def test_native_round_loop_one_rank_failure_fails_every_rank(kind, top):
    """a failure only one rank sees (here rank 1's done buffer is too small) is carried by
    the next collective, so every rank returns an error from the same call -- none blocks in a
    collective the failed rank never joins.  The threads join within the timeout, all with errors."""
    import threading
    from oversim_amd import Params
    from oversim_amd.shard import (GpuShardStepper, KadShardStepper, arc_bounds, local_exchanges, native_kad_route,
                                   native_route, destroy_exchange)
    world, n, m = 3, 1 << 14, 3000
    net = W.population(n, 0x6A)
    bounds = arc_bounds(n, world)
    dev = torch.device("cuda", 0)
    ks, ss, _, _ = _native_inputs(net, bounds, world, m, 0x6B)
    if kind == "chord":
        steppers = [GpuShardStepper(net.ids, net.xy, bounds, r, dev, capacity=m, top_levels=top) for r in range(world)]
        for st in steppers:
            st.reset(world * m)
    else:
        params = Params.kademlia().replace(lookupParallelRpcs=3)
        steppers = [KadShardStepper(net.ids, net.xy, bounds, r, dev, params=params, top_levels=top)
                    for r in range(world)]
    exs = local_exchanges(world)
    errs = [None] * world

    def run(r):
        cap = 10 if r == 1 else None
        try:
            with torch.cuda.device(dev):
                if kind == "chord":
                    native_route(steppers[r], exs[r], ks[r], ss[r], r * m, cohorts=2, done_cap=cap)
                else:
                    native_kad_route(steppers[r], exs[r], ks[r], ss[r], r * m, done_cap=cap)
        except Exception as e:       # noqa: BLE001
            errs[r] = e

    th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in th), "a rank is still blocked in a collective"
    assert all(e is not None for e in errs), errs
    assert "done" in str(errs[1]) or "done_cap" in str(errs[1]), errs[1]
    for ex in exs:
        destroy_exchange(ex)
    # the contexts stay usable: the same batch with room for it routes
    if kind == "chord":
        res = [None] * world

        def ok(r):
            with torch.cuda.device(dev):
                res[r] = native_route(steppers[r], exs2[r], ks[r], ss[r], r * m, cohorts=2)

        exs2 = local_exchanges(world)
        th = [threading.Thread(target=ok, args=(r,)) for r in range(world)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=120)
        assert sum(int(x[0].shape[0]) for x in res) == world * m
        for ex in exs2:
            destroy_exchange(ex)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["chord", "kademlia"])
def test_native_round_loop_rccl_world1(kind):
    """The library's own RCCL exchange (ovs_rccl_unique_id + ovs_exchange_rccl_create, one
    communicator of one rank on this box): the sharded route at W = 1 through RCCL equals the
    single-context route (the W > 1 path differs only in the peers of the send/recv group)."""
    from oversim_amd import Params
    from oversim_amd.shard import (GpuShardStepper, KadShardStepper, arc_bounds, done_to_numpy, destroy_exchange,
                                   native_kad_route, native_route, rccl_exchange, rccl_unique_id)
    n, m = 1 << 15, 20000
    net = W.population(n, 0x5C)
    bounds = arc_bounds(n, 1)
    ks, ss, allk, alls = _native_inputs(net, bounds, 1, m, 0x5D, node_ids=lambda r: False)
    dev = torch.device("cuda", 0)
    ex = rccl_exchange(0, 1, 0, rccl_unique_id())
    try:
        if kind == "chord":
            st = GpuShardStepper(net.ids, net.xy, bounds, 0, dev, capacity=m)
            st.reset(m)
            done, stats = native_route(st, ex, ks[0], ss[0], 0, cohorts=2)
            ref = _single_gpu_reference(net, allk, alls)
        else:
            params = Params.kademlia().replace(lookupParallelRpcs=3)
            st = KadShardStepper(net.ids, net.xy, bounds, 0, dev, params=params)
            done, stats = native_kad_route(st, ex, ks[0], ss[0], 0)
            ref = _kad_reference(net, allk, alls, params)
    finally:
        destroy_exchange(ex)
    d = done_to_numpy(done)
    d = d[np.argsort(d["qid"])]
    assert np.array_equal(d["qid"], np.arange(m))
    for f in ROUTE_FIELDS:
        assert np.array_equal(d[f].astype(np.int64), ref[f].astype(np.int64)), f
    assert stats.rounds >= 1 and stats.sent == 0


def _native_gloo_worker(rank, world, port, q, kind):
    import traceback
    try:
        _native_gloo_body(rank, world, port, q, kind)
    except BaseException:       # noqa: BLE001 -- reported to the parent, which stops the other rank
        q.put(("error", rank, traceback.format_exc()))
        raise


def _native_gloo_body(rank, world, port, q, kind):
    import torch.distributed as dist
    from oversim_amd import Params
    from oversim_amd.shard import (CallbackExchange, GpuShardStepper, KadShardStepper, arc_bounds, done_to_numpy,
                                   native_kad_route, native_route)
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n, m = 1 << 14, 3000
    net = W.population(n, 0x5E)
    bounds = arc_bounds(n, world)
    k, s = W.lookups(net.ids, m, 0x5F + rank, node_ids=False)
    s = (bounds[rank] + s.astype(np.int64) % (bounds[rank + 1] - bounds[rank])).astype(np.uint32)
    dev = torch.device("cuda", 0)
    kt, st_ = torch.from_numpy(k.view(np.int32)).to(dev), torch.from_numpy(s.view(np.int32)).to(dev)
    cx = CallbackExchange(dev)
    if kind == "chord":
        st = GpuShardStepper(net.ids, net.xy, bounds, rank, dev, capacity=m)
        st.reset(world * m)
        done, stats = native_route(st, cx.ex, kt, st_, rank * m, cohorts=2)
    else:
        # kademlia_mig: replicated top buckets, the one-way lookups migrate between the two processes
        st = KadShardStepper(net.ids, net.xy, bounds, rank, dev, params=Params.kademlia(),
                             top_levels=3 if kind == "kademlia_mig" else 0)
        done, stats = native_kad_route(st, cx.ex, kt, st_, rank * m)
    q.put((rank, done_to_numpy(done), k, s, int(stats.rounds)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["chord", "kademlia", "kademlia_mig"])
def test_native_round_loop_gloo_two_processes(kind):
    """The native loop over a caller-supplied exchange: Python callbacks running torch.distributed
    gloo collectives (CallbackExchange), two processes sharing the GPU."""
    import torch.multiprocessing as mp
    from oversim_amd import Params
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_native_gloo_worker, args=(r, world, port, q, kind)) for r in range(world)]
    for p in procs:
        p.start()
    res = []
    try:
        for _ in range(world):
            x = q.get(timeout=150)
            if x[0] == "error":
                pytest.fail(f"rank {x[1]} failed:\n{x[2]}")
            res.append(x)
    finally:
        if len(res) < world:
            for p in procs:       # the surviving rank waits in a collective: stop our own children
                p.kill()
    res.sort(key=lambda x: x[0])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    d = np.concatenate([r[1] for r in res])
    d = d[np.argsort(d["qid"])]
    m = 3000
    assert np.array_equal(d["qid"], np.arange(world * m))
    net = W.population(1 << 14, 0x5E)
    keys, src = np.concatenate([r[2] for r in res]), np.concatenate([r[3] for r in res])
    ref = _single_gpu_reference(net, keys, src) if kind == "chord" else _kad_reference(net, keys, src, Params.kademlia())
    # (kademlia_mig: lookups that migrate finish on either rank; the qids cover the batch once)
    for f in ROUTE_FIELDS:
        assert np.array_equal(d[f].astype(np.int64), ref[f].astype(np.int64)), f


# ------------------------------------------------- Kademlia lookups that migrate (ABI 11)

@pytest.mark.gpu
@pytest.mark.parametrize("world,alpha,n,top", [(2, 3, 1 << 16, 3), (8, 3, 1 << 16, 3), (3, 1, 15000, 2), (4, 8, 1 << 16, 4),
                                               (3, 3, 15000, 0), (8, 2, 3000, 7), (5, 3, 1 << 16, 1)])
def test_kad_migration_emulated_on_one_gpu(world, alpha, n, top):
    """Kademlia one-way lookups that move between arcs (ovs_kad_shard_mig_step; W contexts on one GPU,
    the in-process exchange): the top `top` buckets of every node replicated, a lookup moved as one
    record to the owner of the rows its next findNode needs.  Every lookup -- responsible node, hops,
    status, latency and its FindNodeCall count -- equals the single-context K2's, including networks
    whose top buckets are not full (3000 nodes, 7 levels) and no replication at all (top 0)."""
    from oversim_amd import Params
    from oversim_amd.shard import KadMigStepper, arc_bounds, done_to_numpy, route_local_shards
    m = 4000
    net = W.population(n, 0x7A + world + alpha)
    bounds = arc_bounds(n, world)
    dev = torch.device("cuda", 0)
    params = Params.kademlia().replace(lookupParallelRpcs=alpha)
    steppers = [KadMigStepper(net.ids, net.xy, bounds, r, dev, params=params, top_levels=top, capacity=world * m)
                for r in range(world)]
    ks, ss, allk, alls = _native_inputs(net, bounds, world, m, 0x7B, node_ids=lambda r: r % 2 == 1)
    dones, rounds = route_local_shards(steppers, ks, ss, [r * m for r in range(world)])
    d = np.concatenate([done_to_numpy(x) for x in dones])
    d = d[np.argsort(d["qid"])]
    assert np.array_equal(d["qid"], np.arange(world * m))
    ref = _kad_reference(net, allk, alls, params)
    for f in ROUTE_FIELDS:
        assert np.array_equal(d[f].astype(np.int64), ref[f].astype(np.int64)), f
    assert np.array_equal(d["pad"].astype(np.int64), ref["rpcs"].astype(np.int64))
    assert rounds >= 2


@pytest.mark.gpu
def test_kad_migration_moves_once_on_prefix_arcs():
    """On arcs cut at key prefixes (W = 8: the top three ID bits) with 3 replicated levels, every
    findNode a lookup needs is either answerable from the replicated top buckets or on its key's arc:
    a lookup moves at most once, so every round after the second is empty."""
    from oversim_amd import Params
    from oversim_amd.shard import KadMigStepper, done_to_numpy, route_local_shards, prefix_bounds
    world, n, m = 8, 1 << 16, 4000
    net = W.population(n, 0x7C)
    bounds = prefix_bounds(net.ids, world)
    dev = torch.device("cuda", 0)
    params = Params.kademlia().replace(lookupParallelRpcs=3)
    steppers = [KadMigStepper(net.ids, net.xy, bounds, r, dev, params=params, top_levels=3, capacity=world * m)
                for r in range(world)]
    ks, ss, allk, alls = _native_inputs(net, bounds, world, m, 0x7D, node_ids=lambda r: False)
    dones, rounds = route_local_shards(steppers, ks, ss, [r * m for r in range(world)])
    assert rounds <= 2, rounds          # round 1 at home, round 2 at the key's arc, nothing left after
    d = np.concatenate([done_to_numpy(x) for x in dones])
    d = d[np.argsort(d["qid"])]
    ref = _kad_reference(net, allk, alls, params)
    for f in ROUTE_FIELDS:
        assert np.array_equal(d[f].astype(np.int64), ref[f].astype(np.int64)), f
