#!/usr/bin/env python3
"""Benchmark: routed lookup hops/s of the MI355X Chord iterative-lookup engine.

Contract (driver): `python bench.py --gpus N --steps K --warmup W`, one process
per GPU (torch.distributed.run for N > 1).  A *step* is one pass of the hot
path over one batch of synthetic lookups resident in HBM: config C of
BASELINE.json -- Chord ring of 2^20 nodes (random coordinates, fieldSize 150),
10M uniform random-key one-way KBR lookups, iterative routing, successor list
8, hopCountMax 50.  Prints ONE JSON line on rank 0.

Multi-GPU: each rank owns one 2^20-node arc of an N x 2^20 ring and originates
10M lookups (weak scaling); lookups whose next responder lies on another arc
are exchanged every hop round with an RCCL all-to-allv.
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

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s
B_HOP = 512                    # algorithmic bytes per Chord hop


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--nodes", type=int, default=1 << 20, help="ring nodes per GPU")
    ap.add_argument("--lookups", type=int, default=10_000_000, help="lookups per GPU per step")
    ap.add_argument("--seed", type=int, default=0xC)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample time")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic-csv", default=None, help="rocprofv3 --pmc counter_collection.csv for `traffic`")
    return ap.parse_args()


def cpu_baseline(ids, xy, keys, src, target_s: float) -> dict:
    """The oracle (CPU restatement, kind 'port') on a bounded sample of the same workload."""
    sys.path.insert(0, str(ROOT / "tests"))
    from oracle_lib import OracleNet
    nthreads = min(os.cpu_count() or 1, 16)
    o = OracleNet("chord", ids, xy)
    m = 20000
    t = time.perf_counter()
    r = o.route(keys[:m], src[:m], record_hops=False, nthreads=nthreads)
    dt = time.perf_counter() - t
    m2 = int(min(len(keys), max(m, m * target_s / max(dt, 1e-6))))
    t = time.perf_counter()
    r = o.route(keys[:m2], src[:m2], record_hops=False, nthreads=nthreads)
    dt = time.perf_counter() - t
    hops = int(r["hops"].astype(np.int64).sum())
    return {"value": hops / dt, "unit": "hops/s", "cores": nthreads, "kind": "port",
            "sample": f"oracle/ovs_oracle.c restatement, {m2} of the step's lookups on the same "
                      f"{len(ids)}-node ring, OpenMP {nthreads} threads, {dt:.1f} s",
            "lookups_per_s": m2 / dt}


def traffic_from_csv(path: str | None, kernel_substr: str = "k_chord_route"):
    if not path or not Path(path).exists():
        return None
    import csv
    tot, n = {}, {}
    with open(path) as f:
        for row in csv.DictReader(f):
            if kernel_substr not in row.get("Kernel_Name", ""):
                continue
            c = row.get("Counter_Name")
            tot[c] = tot.get(c, 0.0) + float(row.get("Counter_Value", 0))
            n[c] = n.get(c, 0) + 1
    if not tot:
        return None
    # FETCH_SIZE / WRITE_SIZE are in KB (x1024); gfx950 FETCH_SIZE counts 128-B requests
    # as 64 B (MI355X_MICROARCH.md §HBM) -> x2 on the read side
    fetch = 2 * 1024 * tot.get("FETCH_SIZE", 0.0) / max(n.get("FETCH_SIZE", 1), 1)
    write = 1024 * tot.get("WRITE_SIZE", 0.0) / max(n.get("WRITE_SIZE", 1), 1)
    return fetch + write


def main():
    a = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from oversim_amd import KbrEngine, Params, workload as W

    nodes_total = a.nodes * world
    ids = W.sorted_unique_ids(nodes_total, a.seed)
    xy = W.coordinates(nodes_total, a.seed, use_file=False)
    keys, src = W.lookups(ids, a.lookups, a.seed + 1000 + rank, node_ids=False)
    if world > 1:
        # lookups originate on this rank's arc
        lo, hi = rank * nodes_total // world, (rank + 1) * nodes_total // world
        src = (lo + (src.astype(np.int64) % (hi - lo))).astype(np.uint32)

    dev = torch.device("cuda", local)
    stream = torch.cuda.Stream(device=dev)
    if world == 1:
        eng = KbrEngine(local)
        eng.set_params(Params.chord())
        eng.chord_load(ids, xy)
        dkeys = torch.from_numpy(keys).to(dev)
        dsrc = torch.from_numpy(src).to(dev)
        dout = torch.empty((a.lookups, 16), dtype=torch.uint8, device=dev)

        def step():
            eng.lookup_device(dkeys.data_ptr(), dsrc.data_ptr(), a.lookups, dout.data_ptr(), stream.cuda_stream)
    else:
        from oversim_amd.shard import ShardedChord
        sh = ShardedChord(rank, world, ids, xy, keys, src, dev, stream)

        def step():
            sh.run()

    torch.cuda.synchronize()
    torch.cuda.set_stream(stream)        # every launch of the step is ordered on `stream`
    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
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
    kern_ms = ev0.elapsed_time(ev1) / max(a.steps, 1)

    # hops of one step (identical every step: same inputs)
    if world == 1:
        outs = dout.cpu().numpy().view(np.uint8).reshape(-1, 16)
        hops = outs[:, 4:6].copy().view(np.uint16).ravel().astype(np.int64)
        status = outs[:, 6]
        n_ok = int((status == 0).sum())
        hop_total = int(hops.sum())
    else:
        hop_total, n_ok = sh.hop_total(), sh.ok_total()

    t = torch.tensor([wall, float(hop_total), float(n_ok)], dtype=torch.float64, device=dev)
    if world > 1:
        w = t[:1].clone()
        dist.all_reduce(w, op=dist.ReduceOp.MAX)
        s = t[1:].clone()
        dist.all_reduce(s, op=dist.ReduceOp.SUM)
        wall_max, hop_all, ok_all = float(w[0]), float(s[0]), float(s[1])
    else:
        wall_max, hop_all, ok_all = wall, float(hop_total), float(n_ok)

    if rank == 0:
        value = hop_all * a.steps / wall_max
        achieved = (hop_total * B_HOP) / (kern_ms * 1e-3) / 1e9
        traffic = traffic_from_csv(a.traffic_csv)
        cpu = None
        if world == 1 and not a.no_cpu_baseline:
            cpu = cpu_baseline(ids, xy, keys, src, a.cpu_seconds)
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
            "dtype": "u32 keys (160-bit int), int64 ns, fp64 coords",
            "data": "synthetic: seeded uniform 160-bit node IDs and keys, uniform(-75,75) coordinates",
            "config": {
                "workload": "C: Chord 2^20 nodes per GPU, 10M random-key iterative one-way lookups per GPU",
                "overlay": "chord", "nodes_per_gpu": a.nodes, "nodes_total": nodes_total,
                "lookups_per_gpu": a.lookups, "successorListSize": 8, "hopCountMax": 50,
                "parallelism": f"ring sharded over {world} GPU(s)",
                "lookups_per_s": ok_all * a.steps / wall_max,
                "mean_hops": hop_all / max(ok_all, 1),
            },
            "roofline": {
                "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": (traffic / 1.0) if traffic else None,
                "kernel": "k_chord_route", "kernel_ms": kern_ms,
                "bytes_per_hop_algorithmic": B_HOP,
            },
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
