#!/usr/bin/env python3
"""Benchmark: routed lookup hops/s of the MI355X KBR lookup engine (BASELINE.json).

Contract (driver): `python bench.py --gpus N --steps K --warmup W`, one process
per GPU (torch.distributed.run for N > 1).  A *step* is one pass of the hot
path over one batch of synthetic lookups already resident in HBM.  rank 0
prints ONE JSON line.

Workloads (--workload, default C):
  A  Chord, 1000 nodes (nodes_2d_15000.xml coordinates), successorListSize 8,
     100k node-ID one-way lookups per GPU, seed 0x4213 (BASELINE.md §2 config
     A, the reference's own CPU-sized case).  N > 1: independent replicas.
  C  Chord, 2^20 ring nodes per GPU (random coordinates, fieldSize 150), 10M
     uniform random-key one-way lookups per GPU.  N > 1: the N x 2^20 ring is
     sharded over the GPUs and in-flight lookups are exchanged every hop round
     with an RCCL all-to-allv (oversim_amd/shard.py).  Weak scaling.
  D  Chord, 2^26-node ring (config D), 8M random-key lookups per GPU, ring
     sharded over the N GPUs (RCCL all-to-allv).  Weak scaling in lookups.
  B  Kademlia, 15 000 nodes (nodes_2d_15000.xml coordinates), k=8, alpha=1,
     1M node-ID lookups per GPU.  N > 1: independent replicas.
  K  Koorde, 2^20 nodes, 4M random-key lookups per GPU (not a BASELINE config:
     the Koorde routing rule).  N > 1: independent replicas.
  R  Kademlia, 2^20 nodes, alpha=3: the bucket refresh (Kademlia.cc:1591-1686,
     exhaustiveRefresh) of 2^16 nodes per GPU, ~1.1M exhaustive-iterative
     lookups with bucketRefreshNodes = 8.  Replicas.
  E  Kademlia, 2^24 nodes, alpha=3, 4M random-key lookups per GPU.  N > 1: the
     ID space is cut into N arcs (prefixes), each GPU owns its arc's tables, and
     FindNodeCalls are exchanged as request/response all-to-allv rounds
     (oversim_amd/shard.py).  Weak scaling in lookups.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

# the 16 B per-lookup result records (include/ovs_kbr.h ovs_route_out / ovs_lookup_out)
ROUTE_DTYPE = np.dtype([("responsible", "<u4"), ("hops", "<u2"), ("status", "u1"),
                        ("one_way_hops", "u1"), ("latency_ns", "<i8")])
LOOKUP_DTYPE = np.dtype([("num_siblings", "<u4"), ("hops", "<u2"), ("status", "u1"),
                         ("is_valid", "u1"), ("latency_ns", "<i8")])

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s
# measured ceiling of dependent random 64 B line gathers from an HBM-resident table (cooperative
# 16 B-per-lane loads, tools/ubench/gather.hip, profiles/r01_j_coop/ubench.txt): 3.9e10-4.7e10 lines/s
GATHER_CEILING_GBS = 2950.0
GATHER_CEILING_LINES = 4.6e10
# Algorithmic bytes.  Chord, converged-ring layout of this build: every hop reads
# the responder's 64 B header line (the finger entry that selected it, or its NodeRec), every
# lookup additionally its source's NodeRec (64 B) and its key/source/result (24 B in, 16 B out).
# SURVEY.md §8(d) priced 512 B/hop for a 24 B-record layout with separate window, finger and
# coordinate gathers; that figure is reported beside ("survey_model", with the fraction it would imply), not used.
B_HOP, B_LOOKUP = 64, 104
B_HOP_SURVEY = 512
# Kademlia, this build's layout: every FindNodeCall reads its target's 64 B KadNode line when it is
# sent and the responder's 96 B bucket block (findNode's main bucket) when its response is
# processed; every lookup additionally its source's KadNode + block (the local findNode at start)
# and its key/source/result (24 B in, 16 B out).  Blocks findNode reads beyond the main bucket
# (short buckets, the sibling zone) are extra, not counted.  SURVEY.md §8(d) priced 448 B/RPC for
# a 24 B-entry layout; reported beside ("survey_model").
B_RPC, B_KLOOKUP = 160, 200
B_RPC_SURVEY = 448
# Koorde: a hop reads the responder's ring records (predecessor, itself, first successor: 3 x 24 B),
# its 16 B KoordeNode and its 16 B coordinates; a lookup its key/source (24 B), the source's
# coordinates (16 B) and writes 16 B.  The successor / de Bruijn list searches are extra.
B_KHOP, B_KLOOKUP_K = 104, 56


def survey_model(kind, hops, rpcs, lookups, kern_ms) -> dict:
    """SURVEY.md §8(d) priced the path for a 24 B-record layout with separate window / finger /
    coordinate gathers (512 B/hop, 448 B/RPC).  This layout moves a fraction of that,
    so the survey model's implied fraction is printed for reference only: above 1 it is physically
    impossible and shows the model is superseded, not that the kernel beats HBM."""
    b = B_HOP_SURVEY * hops if kind == "chord" else B_RPC_SURVEY * (rpcs or 0)
    f = b / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS
    return {"bytes_per_unit": B_HOP_SURVEY if kind == "chord" else B_RPC_SURVEY, "implied_frac": f,
            "note": "SURVEY §8(d) layout model, superseded by this build's layout (DESIGN.md §5); not the roofline"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", choices=["A", "B", "C", "D", "E", "K", "R"], default="C")
    ap.add_argument("--nodes", type=int, default=None, help="override ring size (per GPU for C, total for D/E)")
    ap.add_argument("--lookups", type=int, default=None, help="override lookups per GPU per step")
    ap.add_argument("--routing", choices=["iterative", "semi-recursive"], default="iterative",
                    help="Chord routingType (semi-recursive = omnetpp.ini ChordLarge)")
    ap.add_argument("--seed", type=int, default=None, help="population seed (default: the workload's, 0xC)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample time")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic-json", default=None,
                    help="PMC summary (tools/pmc_json.py); default profiles/pmc/<workload>.json when present")
    ap.add_argument("--traffic-csv", default=None,
                    help="rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE outputs (counter_collection.csv or run_results.db), "
                         "comma separated")
    return ap.parse_args()


def cpu_baseline(kind, ids, xy, keys, src, target_s: float, alpha: int = 1, routing_type: int = 0,
                 refresh_R: int = 0) -> dict:
    """The oracle (CPU restatement, kind 'port', built -O3) on a bounded sample of the same workload,
    timed on all the host cores this job may use and on one core.  Populations too large for the
    oracle's stored tables (configs D, E) use its lazy tables (every table entry evaluated per
    access), which makes that port slower than one holding the tables."""
    sys.path.insert(0, str(ROOT / "tests"))
    from oracle_lib import OracleNet, chord_params, kad_params, koorde_params
    nproc = os.cpu_count() or 1
    # the job's CPU share: OMP_NUM_THREADS on the GPU box (16 per GPU), else every CPU
    nthreads = max(1, min(nproc, int(os.environ.get("OMP_NUM_THREADS", nproc))))
    lazy = len(ids) > (1 << 22)
    if kind == "koorde":
        o = OracleNet(kind, ids, xy, koorde_params())
    else:
        o = OracleNet(kind, ids, xy, kad_params(lookupParallelRpcs=alpha) if kind == "kademlia"
                      else chord_params(routingType=routing_type), lazy=lazy)

    def run(m, threads):
        if refresh_R:
            return o.exhaustive(keys[:m], src[:m], refresh_R, record=False, nthreads=threads)
        return o.route(keys[:m], src[:m], record_hops=False, count_rpcs=kind == "kademlia", nthreads=threads)

    def timed(threads: int, budget_s: float):
        # calibrate on growing prefixes until one takes a quarter of the budget (a short probe
        # is dominated by thread start-up and would undersize the sample), then run the sample
        m = 2000
        while True:
            t = time.perf_counter()
            run(m, threads)
            dt = time.perf_counter() - t
            if dt >= 0.25 * budget_s or m >= len(keys):
                break
            m = min(len(keys), m * max(2, int(0.25 * budget_s / max(dt, 1e-6))))
        m2 = int(min(len(keys), max(m, m * budget_s / max(dt, 1e-6))))
        t = time.perf_counter()
        r = run(m2, threads)
        dt = time.perf_counter() - t
        return int(r["hops"].astype(np.int64).sum()) / dt, m2 / dt, m2, dt, r

    hps, lps, m_all, dt_all, res = timed(nthreads, target_s)
    hps1, lps1, m_one, dt_one, _ = timed(1, target_s / 2)
    return {"value": hps, "unit": "hops/s", "cores": nthreads, "kind": "port",
            "sample": f"oracle/ovs_oracle.c restatement (gcc -O3, OpenMP), {m_all} of the step's lookups on the same "
                      f"{len(ids)}-node {kind} network{' (lazy tables)' if lazy else ''}: {nthreads} threads "
                      f"{dt_all:.1f} s; 1 thread {m_one} lookups {dt_one:.1f} s",
            "lookups_per_s": lps, "host_cpus": nproc, "value_1core": hps1, "lookups_per_s_1core": lps1}, res


# output fields the parity check compares, per result kind (the oracle's record dtypes, tests/oracle_lib.py):
# one-way route -> ovs_route_out (IterativeLookup getResult()[0] / getMinHops(), BaseOverlay.cc:1241-1307 +
# the route message's latency); refresh lookups -> ovs_lookup_out + the R-node result + FindNodeCall counts
ROUTE_FIELDS = ("responsible", "hops", "status", "one_way_hops", "latency_ns")
LOOKUP_FIELDS = ("num_siblings", "hops", "status", "is_valid", "latency_ns")


def parity_check(gpu: dict, orc: dict, m: int, fields) -> dict:
    """Field-by-field comparison of the step's GPU results with the CPU oracle's on the first m lookups of
    the same batch (the lookups cpu_baseline() ran).  Every field must be equal (bit-exact contract,
    latency in int64 ns)."""
    bad = np.zeros(m, dtype=bool)
    per = {}
    for f in fields:
        a, b = np.asarray(gpu[f])[:m], np.asarray(orc[f])[:m]
        d = a != b
        if d.ndim > 1:
            d = d.reshape(m, -1).any(axis=1)
        per[f] = int(d.sum())
        bad |= d
    out = {"checked": int(m), "mismatches": int(bad.sum()), "fields": list(fields),
           "per_field": per, "reference": "oracle/ovs_oracle.c (CPU restatement, the cpu_baseline run's own results)"}
    if bad.any():
        out["first_mismatch"] = int(np.argmax(bad))
    return out


class Watchdog:
    """Ends a stuck run instead of letting it block the job: when the current stage has not moved on
    within its limit, the stage -- and, inside the native round loop, the collective it is in
    (ovs_exchange_stage) -- goes to stderr and the process exits 124.  A collective that hangs on one
    rank thus fails every rank's job with a named stage (init, warmup, timed step, count allgather,
    records alltoallv, completeness allreduce, parity gather, ...)."""

    def __init__(self, rank: int):
        import threading
        self.rank = rank
        self.scale = float(os.environ.get("OVS_BENCH_STAGE_SCALE", "1.0"))
        self.stage, self.limit, self.t = "start", 600.0, time.monotonic()
        threading.Thread(target=self._run, daemon=True).start()

    def set(self, stage: str, limit: float):
        self.stage, self.limit, self.t = stage, limit * self.scale, time.monotonic()

    def _run(self):
        while True:
            time.sleep(2.0)
            if time.monotonic() - self.t > self.limit:
                inner = ""
                try:
                    import ctypes as C
                    from oversim_amd.kbr import lib
                    f = lib().ovs_exchange_stage
                    f.argtypes, f.restype = [C.POINTER(C.c_uint32)], C.c_char_p
                    rnd = C.c_uint32(0)
                    inner = f" (round loop: {f(C.byref(rnd)).decode()}, round {rnd.value})"
                except Exception:       # noqa: BLE001
                    pass
                sys.stderr.write(f"bench.py rank {self.rank}: stage '{self.stage}' stuck for more than "
                                 f"{self.limit:.0f} s{inner}; exiting\n")
                sys.stderr.flush()
                os._exit(124)


# lookups of each rank's batch the N > 1 line checks against the oracle (lazy tables above 2^22 nodes)
PARITY_SAMPLE = {"C": 50_000, "D": 20_000, "E": 10_000}


def sharded_parity(sh, kind, ids, xy, keys_t, src_t, m, world, comm_dev, sample, alpha, routing_type) -> dict:
    """The N > 1 line's correctness evidence.  Lookups migrate, so a lookup's done record lives on the
    rank where it finished: every rank takes the records it holds of the first `sample` lookups of any
    rank's batch (qid = home rank x m + index), routes those same (key, source) pairs through the CPU
    oracle -- the checker cpu_baseline() uses -- and compares every field; the counts are summed over
    the ranks, so each sampled lookup is checked exactly once, wherever it finished."""
    import torch
    import torch.distributed as dist
    from oversim_amd.shard import done_to_numpy
    sys.path.insert(0, str(ROOT / "tests"))
    from oracle_lib import OracleNet, chord_params, kad_params
    S = int(min(sample, m))
    kk, ss = keys_t[:S].contiguous().to(comm_dev), src_t[:S].contiguous().to(comm_dev)
    gk = [torch.empty_like(kk) for _ in range(world)]
    gs = [torch.empty_like(ss) for _ in range(world)]
    dist.all_gather(gk, kk)
    dist.all_gather(gs, ss)
    K = torch.stack(gk).cpu().numpy().view(np.uint32).reshape(world, S, 5)
    Sr = torch.stack(gs).cpu().numpy().view(np.uint32).reshape(world, S)
    d = done_to_numpy(sh._done)
    q = d["qid"].astype(np.int64)
    home, idx = q // m, q % m
    sel = idx < S
    keys, src = np.ascontiguousarray(K[home[sel], idx[sel]]), np.ascontiguousarray(Sr[home[sel], idx[sel]])
    fields = ROUTE_FIELDS + (("rpcs",) if kind == "kademlia" else ())
    per = np.zeros(len(fields), dtype=np.int64)
    bad = 0
    if len(keys):
        o = OracleNet(kind, ids, xy, kad_params(lookupParallelRpcs=alpha) if kind == "kademlia"
                      else chord_params(routingType=routing_type), lazy=len(ids) > (1 << 22))
        nthreads = max(1, min(os.cpu_count() or 1, int(os.environ.get("OMP_NUM_THREADS", "16"))))
        r = o.route(keys, src, record_hops=False, count_rpcs=kind == "kademlia", nthreads=nthreads)
        got = {f: d[f][sel] for f in ROUTE_FIELDS}
        if kind == "kademlia":
            got["rpcs"] = d["pad"][sel]
        wrong = np.zeros(len(keys), dtype=bool)
        for i, f in enumerate(fields):
            x = np.asarray(got[f]).astype(np.int64) != np.asarray(r[f]).astype(np.int64)
            per[i] = int(x.sum())
            wrong |= x
        bad = int(wrong.sum())
    t = torch.tensor([len(keys), bad] + per.tolist(), dtype=torch.int64, device=comm_dev)
    dist.all_reduce(t)
    t = t.cpu().tolist()
    return {"checked": int(t[0]), "expected": world * S, "mismatches": int(t[1]), "fields": list(fields),
            "per_field": dict(zip(fields, (int(x) for x in t[2:]))), "sample_per_rank": S,
            "reference": "oracle/ovs_oracle.c (CPU restatement) on each rank's held done records of the sample"
                         + (" (lazy tables)" if len(ids) > (1 << 22) else "")}


def traffic_from_json(path: str | None, workload: str, kname: str):
    """HBM bytes per launch of the dominant kernel from a committed PMC summary
    (profiles/pmc/<workload>.json, written by tools/pmc_json.py from rocprofv3 --pmc FETCH_SIZE and
    WRITE_SIZE passes of this same workload).  FETCH_SIZE counts the random 64 B line gathers of
    these kernels at 64 B each -- calibrated on tools/ubench/gather.hip with a known byte count
    (profiles/r01_j_coop/calib.txt) -- so no x2 correction is applied."""
    p = Path(path) if path else ROOT / "profiles" / "pmc" / f"{workload}.json"
    if not p.exists():
        return None, None
    d = json.loads(p.read_text())
    if kname not in d.get("kernel", ""):
        return None, None
    return 1024.0 * (d["fetch_kb"] + d["write_kb"]), str(p.relative_to(ROOT) if p.is_absolute() and ROOT in p.parents else p)


def traffic_from_csv(path: str | None, kernel_substr: str):
    """HBM bytes per launch from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs (KB units;
    gfx950 FETCH_SIZE tallies 128-B requests as 64 B -> x2 on the read side, MI355X_MICROARCH.md §HBM).
    Accepts rocprofv3 counter_collection.csv files or its SQLite run_results.db files, comma separated."""
    if not path:
        return None
    import csv
    import sqlite3
    tot, n = {}, {}

    def add(kernel, counter, value):
        if kernel_substr not in kernel:
            return
        tot[counter] = tot.get(counter, 0.0) + float(value)
        n[counter] = n.get(counter, 0) + 1

    for p in path.split(","):
        if not Path(p).exists():
            continue
        if p.endswith(".db"):
            c = sqlite3.connect(p)
            try:
                for kname, counter, value in c.execute(
                        "select k.name, e.counter_name, sum(e.counter_value) from pmc_events e join kernels k "
                        "on k.dispatch_id = e.dispatch_id group by e.dispatch_id, e.counter_name"):
                    add(kname, counter, value)
            finally:
                c.close()
        else:
            with open(p) as f:
                for row in csv.DictReader(f):
                    add(row.get("Kernel_Name", ""), row.get("Counter_Name"), row.get("Counter_Value", 0))
    if "FETCH_SIZE" not in tot:
        return None
    fetch = 2 * 1024 * tot["FETCH_SIZE"] / n["FETCH_SIZE"]
    write = 1024 * tot.get("WRITE_SIZE", 0.0) / max(n.get("WRITE_SIZE", 1), 1)
    return fetch + write


def main():
    a = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    wd = Watchdog(rank)
    wd.set("init", 600)
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("OVS_BENCH_BACKEND", "nccl")      # gloo: rehearse N ranks on one GPU
    ndev = torch.cuda.device_count()
    dev_index = local % max(ndev, 1)
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    dist_on = world > 1 or os.environ.get("OVS_BENCH_SHARD") == "1"
    # the JSON line is the only stdout of the run: RCCL prints its version banner to fd 1 when the
    # first communicator comes up, so fd 1 goes to stderr and the line to the saved descriptor
    json_fd = None
    if dist_on:
        sys.stdout.flush()
        json_fd = os.dup(1)
        os.dup2(2, 1)
    if dist_on:
        from datetime import timedelta
        # torch's own collectives (barriers, the result all-reduces) give up after 5 minutes
        tmo = timedelta(seconds=float(os.environ.get("OVS_BENCH_COLLECTIVE_TIMEOUT", "300")))
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev, timeout=tmo)
        else:
            dist.init_process_group(backend, timeout=tmo)

    from oversim_amd import KbrEngine, Params, workload as W

    wl = dict(W.WORKLOADS[a.workload])
    kind = wl["overlay"]
    routing_type = 1 if a.routing == "semi-recursive" else 0
    if routing_type and kind != "chord":
        raise SystemExit("--routing semi-recursive applies to the Chord workloads (C, D)")
    if routing_type:
        wl["desc"] = wl["desc"].replace("iterative", "semi-recursive")
    stream = torch.cuda.Stream(device=dev)
    # Koorde runs replicas (its tables are not sharded); Kademlia shards unless OVS_KAD_REPLICAS=1
    refresh = a.workload == "R"
    sharded = world > 1 and ((kind == "chord" and a.workload != "A") or (kind == "kademlia" and not refresh and
                                                 os.environ.get("OVS_KAD_REPLICAS") != "1"))
    # rehearsal knob: the sharded host path (collectives, cohorts) at N = 1
    if os.environ.get("OVS_BENCH_SHARD") == "1" and kind != "koorde" and not refresh and a.workload != "A":
        sharded = True

    # ---- population (identical on every rank) and this rank's lookups, resident in HBM
    wd.set("population and table build", 600)
    I = W.bench_inputs(a.workload, dev, world=world, rank=rank, seed=a.seed, nodes=a.nodes, n_lookups=a.lookups,
                       sharded=sharded)
    n_total, m, lo, hi = I["n_total"], I["m"], I["lo"], I["hi"]
    ids_t, xy_t, dkeys, dsrc = I["ids_t"], I["xy_t"], I["keys_t"], I["src_t"]
    ids, xy, keys, src = I["ids"], I["xy"], I["keys"], I["src"]

    # ---- engine
    if sharded:
        from oversim_amd.shard import ShardedChord, ShardedKademlia
        ids_np = ids if ids is not None else ids_t.cpu().numpy().view(np.uint32)
        xy_np = xy if xy is not None else xy_t.cpu().numpy()
        comm = dev if backend == "nccl" else torch.device("cpu")
        if kind == "chord":
            sh = ShardedChord(rank, world, ids_np, xy_np, dkeys, dsrc, dev, comm_dev=comm,
                              params=Params.chord().replace(routingType=routing_type))
            kname = "k_chord_lanes"
        else:
            sh = ShardedKademlia(rank, world, ids_np, xy_np, dkeys, dsrc, dev, comm_dev=comm,
                                 params=Params.kademlia().replace(lookupParallelRpcs=wl["alpha"]))
            kname = "k_kad_route"     # its shard-step instantiation

        def step():
            sh.run()
    else:
        eng = KbrEngine(dev_index)
        if kind == "chord":
            eng.set_params(Params.chord().replace(routingType=routing_type))
            torch.cuda.synchronize()
            eng.chord_load_device(ids_t.data_ptr(), xy_t.data_ptr(), n_total)
            kname = "k_chord_lanes"
        elif kind == "koorde":
            eng.set_params(Params.koorde())
            torch.cuda.synchronize()
            eng.koorde_load_device(ids_t.data_ptr(), xy_t.data_ptr(), n_total)
            kname = "k_koorde_route"
        else:
            eng.set_params(Params.kademlia().replace(lookupParallelRpcs=wl["alpha"]))
            torch.cuda.synchronize()
            eng.kad_load_device(ids_t.data_ptr(), xy_t.data_ptr(), n_total)
            kname = "k_kad_route"
        if refresh:
            # this rank's share of the refresh round: every bucket refresh of its 2^16 nodes
            nn = wl["refresh_nodes"]
            nodes = ((np.arange(nn, dtype=np.int64) * (n_total // nn) + rank) % n_total).astype(np.uint32)
            keys, src = eng.kad_refresh_keys(nodes)
            m = len(keys)
            dkeys = torch.from_numpy(keys.view(np.int32)).to(dev)
            dsrc = torch.from_numpy(src.view(np.int32)).to(dev)
            dsib = torch.empty((m, 8), dtype=torch.int32, device=dev)
            kname = "k_kad_refresh"
        dout = torch.empty((m, 16), dtype=torch.uint8, device=dev)
        drpc = torch.empty(m, dtype=torch.int32, device=dev) if kind == "kademlia" else None

        def step():
            if refresh:
                eng.kad_refresh_device(dkeys.data_ptr(), dsrc.data_ptr(), m, 8, dout.data_ptr(), dsib.data_ptr(),
                                       drpc.data_ptr(), stream.cuda_stream)
                return
            eng.lookup_device(dkeys.data_ptr(), dsrc.data_ptr(), m, dout.data_ptr(), stream.cuda_stream,
                              rpcs_ptr=drpc.data_ptr() if drpc is not None else None)

    torch.cuda.synchronize()
    torch.cuda.set_stream(stream)        # every launch of a step is ordered on `stream`
    for i in range(a.warmup):
        wd.set(f"warmup step {i}", 180)
        step()
    torch.cuda.synchronize()
    wd.set("barrier before the timed region", 300)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    wd.set("timed region", 120 + 60 * a.steps)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(a.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    wd.set("results", 300)
    step_ms = ev0.elapsed_time(ev1) / max(a.steps, 1)

    # ---- work of one step (identical every step: same inputs)
    rpc_total = None
    gres = None          # the last step's per-lookup results, in batch order (for the parity check)
    if sharded:
        hop_total, n_ok = sh.hop_total(), sh.ok_total()
        kern_ms = sh.kernel_ms / max(sh.runs, 1)
        if kind == "kademlia":
            rpc_total = sh.rpc_total()     # FindNodeCalls of this rank's lookups (done records)
        if world == 1:
            gres = sh.results_by_qid()
    else:
        outs = dout.cpu().numpy().reshape(-1, 16)
        hop_total = int(outs[:, 4:6].copy().view(np.uint16).astype(np.int64).sum())
        n_ok = int((outs[:, 6] == 0).sum())
        rec = outs.reshape(-1).view(LOOKUP_DTYPE if refresh else ROUTE_DTYPE)
        gres = {f: rec[f] for f in rec.dtype.names}
        if drpc is not None:
            rpcs_np = drpc.cpu().numpy().view(np.uint32)
            rpc_total = int(rpcs_np.astype(np.int64).sum())
            gres["rpcs"] = rpcs_np
        if refresh:
            gres["siblings"] = dsib.cpu().numpy().view(np.uint32)
        kern_ms = step_ms

    sparity = None
    if sharded and world > 1 and os.environ.get("OVS_BENCH_PARITY", "1") != "0":
        wd.set("sharded parity check (oracle)", 900)
        sample = int(os.environ.get("OVS_BENCH_PARITY_SAMPLE", PARITY_SAMPLE.get(a.workload, 20_000)))
        sparity = sharded_parity(sh, kind, ids_np, xy_np, dkeys, dsrc, m, world,
                                 dev if backend == "nccl" else torch.device("cpu"), sample, wl.get("alpha", 1),
                                 routing_type)
        wd.set("results", 300)
    t = torch.tensor([wall, float(hop_total), float(n_ok), float(rpc_total or 0)], dtype=torch.float64, device=dev)
    if world > 1:
        tt = t.to("cpu") if backend != "nccl" else t
        w = tt[:1].clone()
        dist.all_reduce(w, op=dist.ReduceOp.MAX)
        s = tt[1:].clone()
        dist.all_reduce(s, op=dist.ReduceOp.SUM)
        wall_max, hop_all, ok_all, rpc_all = float(w[0]), float(s[0]), float(s[1]), float(s[2])
    else:
        wall_max, hop_all, ok_all, rpc_all = wall, float(hop_total), float(n_ok), float(rpc_total or 0)

    if rank == 0:
        value = hop_all * a.steps / wall_max
        lookups_launch = n_ok
        if kind == "chord":
            per_launch_bytes = hop_total * B_HOP + lookups_launch * B_LOOKUP
            bper = f"{B_HOP} B/hop + {B_LOOKUP} B/lookup"
        elif kind == "koorde":
            per_launch_bytes = hop_total * B_KHOP + lookups_launch * B_KLOOKUP_K
            bper = f"{B_KHOP} B/hop + {B_KLOOKUP_K} B/lookup"
        else:
            per_launch_bytes = rpc_total * B_RPC + lookups_launch * B_KLOOKUP
            bper = f"{B_RPC} B/RPC + {B_KLOOKUP} B/lookup"
        achieved = per_launch_bytes / (kern_ms * 1e-3) / 1e9
        traffic, traffic_src = (traffic_from_json(a.traffic_json, a.workload, kname) if world == 1 and not sharded
                                else (None, None))
        if a.traffic_csv:
            traffic, traffic_src = traffic_from_csv(a.traffic_csv, kname), a.traffic_csv
        cpu = None
        parity = sparity
        if world == 1 and not a.no_cpu_baseline:
            wd.set("cpu baseline", 900)
            if ids is None:       # device-generated population (D, E): the oracle needs host copies
                ids, xy = ids_t.cpu().numpy().view(np.uint32), xy_t.cpu().numpy()
                keys, src = dkeys[:1 << 20].cpu().numpy().view(np.uint32), dsrc[:1 << 20].cpu().numpy().view(np.uint32)
            cpu, orc = cpu_baseline(kind, ids, xy, keys, src, a.cpu_seconds, wl.get("alpha", 1), routing_type,
                                    refresh_R=8 if refresh else 0)
            if gres is not None:
                # the bench checks its own output: the oracle results the baseline just computed against
                # the GPU's on the same lookups, field by field
                mchk = len(orc["hops"])
                if refresh:
                    fields = LOOKUP_FIELDS + ("siblings", "rpcs")
                else:
                    fields = ROUTE_FIELDS + (("rpcs",) if kind == "kademlia" and "rpcs" in gres else ())
                parity = parity_check(gres, orc, mchk, fields)
                parity["of_batch"] = int(m)
        xname = "RCCL" if backend == "nccl" else f"{backend} (rehearsal)"
        cfg = {"workload": wl["desc"], "overlay": kind, "nodes_total": n_total, "lookups_per_gpu": m,
               "hopCountMax": 50,
               "parallelism": ((f"ring sharded over {world} GPUs ({xname} all-to-allv per hop round)" if kind == "chord"
                                else (f"ID arcs over {world} GPUs, lookups migrate between arcs ({xname} all-to-allv "
                                      "per round)") if getattr(sh.stepper, "top_levels", 0)
                                else f"ID arcs over {world} GPUs, FindNodeCall request/response {xname} all-to-allv per round")
                               if sharded else ("replicas" if world > 1 else "1 GPU")),
               "lookups_per_s": ok_all * a.steps / wall_max, "mean_hops": hop_all / max(ok_all, 1),
               "seed": hex(I["seed"])}
        if refresh:
            cfg.update({"refresh_nodes_per_gpu": wl["refresh_nodes"], "bucketRefreshNodes": 8,
                        "routingType": "exhaustive-iterative"})
        if kind == "kademlia":
            cfg.update({"k": 8, "alpha": wl["alpha"], "rpcs_per_s": rpc_all * a.steps / wall_max,
                        "mean_rpcs": rpc_all / max(ok_all, 1)})
        elif kind == "koorde":
            cfg.update({"successorListSize": 16, "deBruijnListSize": 16, "shiftingBits": 4, "routingType": "iterative"})
        else:
            cfg.update({"successorListSize": 8, "routingType": a.routing})
        if sharded:
            cfg.update({"hop_rounds": sh.rounds,
                        "round_loop": "C++ (ovs_shard_route_batch)" if getattr(sh, "native", False) else "python",
                        "shard_stats_rank0": getattr(sh, "stats", None)})
            cfg["replicated_top_levels"] = getattr(sh.stepper, "top_levels", 0)
            if kind == "kademlia":
                cfg["lookups_migrate"] = bool(getattr(sh.stepper, "top_levels", 0))
        line = {
            "metric": "routed lookup hops/sec (whole node)",
            "value": value,
            "unit": "hops/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": wall_max / a.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32 (160-bit keys), int64 ns, fp64 coordinates",
            "data": "synthetic: seeded uniform 160-bit node IDs and keys; coordinates uniform(-75,75) "
                    "or nodes_2d_15000.xml records (B)",
            "config": cfg,
            "roofline": {
                "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "kernel": kname, "kernel_ms": kern_ms,
                "algorithmic_bytes": bper, "unit_of_work": "RPC" if kind == "kademlia" else "hop",
                "traffic_source": traffic_src,
                # the PMC bytes per launch over this run's kernel time: what HBM actually delivered
                "frac_counter": (traffic / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS) if traffic else None,
                # 64 B lines per second the kernel fetched, beside the measured ceiling of dependent
                # random 64 B gathers (tools/ubench/gather.hip: 4.6e10-4.8e10 lines/s)
                "lines_per_s": (traffic / 64.0 / (kern_ms * 1e-3)) if traffic else None,
                "gather_ceiling_lines_per_s": GATHER_CEILING_LINES,
                "gather_ceiling_GBs": GATHER_CEILING_GBS,
                "frac_of_gather_ceiling": achieved / GATHER_CEILING_GBS,
                **({"survey_model": survey_model(kind, hop_total, rpc_total, lookups_launch, kern_ms)}
                   if kind in ("chord", "kademlia") else {}),
            },
            "cpu_baseline": cpu,
            "parity": parity,
        }
        if json_fd is not None:
            os.write(json_fd, (json.dumps(line) + "\n").encode())
        else:
            print(json.dumps(line), flush=True)
    wd.set("teardown", 300)
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
