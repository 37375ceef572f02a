"""W = 8 cost model of the sharded paths, emulated on one GPU (eight engine contexts, one per arc,
the in-process exchange of oversim_amd.shard): per round and per arc the step kernel time, the
serve / deliver kernel times (Kademlia), the records each arc sends to the others and the active
lookups -- the inputs of DESIGN.md §6's per-rank estimate for a real 8-GPU node.

usage: python tools/diag/shard_w8_model.py --workload E [--lookups-per-rank M] [--world 8]
Prints one JSON line per round and a summary line."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch

from oversim_amd import Params, workload as W
from oversim_amd.shard import (KAD_REQ_BYTES, KAD_RESP_BYTES, REC_BYTES, GpuShardStepper, KadMigStepper, KadShardStepper,
                               arc_bounds, done_to_numpy, prefix_bounds)

ap = argparse.ArgumentParser()
ap.add_argument("--workload", choices=["C", "D", "E"], required=True)
ap.add_argument("--lookups-per-rank", type=int, default=0)
ap.add_argument("--world", type=int, default=8)
ap.add_argument("--nodes", type=int, default=None,
                help="ring size override (D: 2^26 does not fit eight emulated arcs in one GPU's 288 GB; 2^25 does)")
ap.add_argument("--top-levels", type=int, default=None,
                help="replicated top finger levels (Chord; default shard.default_top_levels) / buckets (Kademlia --mig; default 3)")
ap.add_argument("--mig", action="store_true", help="Kademlia: migrating lookups over replicated top buckets, prefix arcs")
ap.add_argument("--xgmi-gbs", type=float, default=64.0,
                help="sustained GB/s per xGMI link and direction for the exchange estimate (7 links per GPU)")
a = ap.parse_args()
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
Wn = a.world
wl = W.WORKLOADS[a.workload]
m = a.lookups_per_rank or wl["lookups"]
inputs = [W.bench_inputs(a.workload, dev, world=Wn, rank=r, n_lookups=m, sharded=True, nodes=a.nodes) for r in range(Wn)]
I0 = inputs[0]
n = I0["n_total"]
ids = I0["ids"] if I0["ids"] is not None else I0["ids_t"].cpu().numpy().view(np.uint32)
xy = I0["xy"] if I0["xy"] is not None else I0["xy_t"].cpu().numpy()
kad = a.workload == "E"
mig = kad and a.mig
bounds = prefix_bounds(ids, Wn) if mig else arc_bounds(n, Wn)
if mig:
    # the lookups' sources must lie on their rank's prefix arc: remap them into it
    for r, I in enumerate(inputs):
        lo_, hi_ = bounds[r], bounds[r + 1]
        I["src_t"] = (lo_ + (I["src_t"].to(torch.int64) % (hi_ - lo_))).to(torch.int32).contiguous()
params = Params.kademlia().replace(lookupParallelRpcs=wl.get("alpha", 3)) if kad else Params.chord()


def ev():
    return torch.cuda.Event(enable_timing=True)


t_start = time.time()
if mig:
    tl = 3 if a.top_levels is None else a.top_levels
    steppers = [KadMigStepper(ids, xy, bounds, r, dev, params=params, top_levels=tl, capacity=Wn * m) for r in range(Wn)]
    # warm-up: one full first-round step per arc (the staging buffers grow to their final size here,
    # not inside the measured rounds: a 256-lookup warm-up left every arc's first round paying the
    # allocations, +1.6 ms)
    for r in range(Wn):
        steppers[r].step(steppers[r].first_batch(inputs[r]["keys_t"], inputs[r]["src_t"], r * m))
    torch.cuda.synchronize()
    for st in steppers:
        st.reset(Wn * m)
    inbox = [steppers[r].first_batch(inputs[r]["keys_t"], inputs[r]["src_t"], r * m) for r in range(Wn)]
    kad = False          # the record loop below (as Chord's)
elif kad:
    steppers = [KadShardStepper(ids, xy, bounds, r, dev, params=params) for r in range(Wn)]
    for r in range(Wn):
        steppers[r].begin(inputs[r]["keys_t"], inputs[r]["src_t"], r * m)
else:
    # send segments of 1.25 m records per destination (a round's inbox is about m; step() grows them)
    steppers = [GpuShardStepper(ids, xy, bounds, r, dev, capacity=m + m // 4, params=params, top_levels=a.top_levels)
                for r in range(Wn)]
    # warm-up: one full first-round step per arc builds the lazily built NodeRecs / finger entries
    # (a one-time cost of the ring's load, not of a step) and grows the staging buffers to size
    for r in range(Wn):
        steppers[r].reset(Wn * m)
        steppers[r].step(steppers[r].first_batch(inputs[r]["keys_t"], inputs[r]["src_t"], r * m))
    torch.cuda.synchronize()
    for st in steppers:
        st.reset(Wn * m)
    # the first round starts from the keys (ovs_shard_step_keys), as route_sharded
    inbox = [steppers[r].first_batch(inputs[r]["keys_t"], inputs[r]["src_t"], r * m) for r in range(Wn)]
torch.cuda.synchronize()
print(json.dumps(dict(workload=a.workload, world=Wn, nodes=n, lookups_per_rank=m, setup_s=round(time.time() - t_start, 1))),
      flush=True)
rounds, tot = 0, dict(step_ms=np.zeros(Wn), serve_ms=np.zeros(Wn), deliver_ms=np.zeros(Wn), sent=np.zeros(Wn))
per_round = []      # (max step ms over the arcs, max bytes an arc sends) per round: the exchange estimate
while True:
    rounds += 1
    segs, rows, kms = [], [], []
    for r in range(Wn):
        e0, e1 = ev(), ev()
        e0.record()
        if kad:
            sg, counts = steppers[r].step()
        else:
            sg, counts = steppers[r].step(inbox[r])
        e1.record()
        segs.append(sg)
        rows.append(counts[:Wn + 1].cpu().numpy().copy() if kad else counts[:Wn].cpu().numpy().copy())
        kms.append((e0, e1))
    torch.cuda.synchronize()
    step_ms = np.array([x.elapsed_time(y) for x, y in kms])
    M = np.stack(rows)
    if int(M.sum()) == 0:
        # the last round: its step finishes the lookups it received and hands nothing on
        tot["step_ms"] += step_ms
        print(json.dumps(dict(round=rounds, step_ms_max=round(float(step_ms.max()), 3),
                              step_ms_mean=round(float(step_ms.mean()), 3), last=True)), flush=True)
        break
    serve_ms, deliver_ms = np.zeros(Wn), np.zeros(Wn)
    if kad:
        replies = [[None] * Wn for _ in range(Wn)]
        for d in range(Wn):
            parts = [segs[r][d][:int(M[r, d])] for r in range(Wn)]
            rows_d = torch.cat(parts)
            if rows_d.shape[0] == 0:
                continue
            e0, e1 = ev(), ev()
            e0.record()
            resp = steppers[d].serve(rows_d)
            e1.record()
            torch.cuda.synchronize()
            serve_ms[d] = e0.elapsed_time(e1)
            off = 0
            for r in range(Wn):
                k = int(M[r, d])
                replies[r][d] = resp[off:off + k]
                off += k
        for r in range(Wn):
            parts = [x for x in replies[r] if x is not None and x.shape[0]]
            if parts:
                e0, e1 = ev(), ev()
                e0.record()
                steppers[r].deliver(torch.cat(parts))
                e1.record()
                torch.cuda.synchronize()
                deliver_ms[r] = e0.elapsed_time(e1)
        # remote requests out (32 B) and their responses back (104 B), per requesting arc
        remote = np.array([int(M[r, :Wn].sum() - M[r, r]) for r in range(Wn)])
        bytes_out = remote * (KAD_REQ_BYTES + KAD_RESP_BYTES)
    else:
        new_inbox = []
        for d in range(Wn):
            parts = [segs[r][d][:int(M[r, d])] for r in range(Wn)]
            new_inbox.append(torch.cat(parts) if parts else segs[d][d][:0])
        inbox = new_inbox
        remote = np.array([int(M[r, :Wn].sum() - M[r, r]) for r in range(Wn)])
        bytes_out = remote * getattr(steppers[0], "rec_bytes", REC_BYTES)
    tot["step_ms"] += step_ms
    tot["serve_ms"] += serve_ms
    tot["deliver_ms"] += deliver_ms
    tot["sent"] += bytes_out
    per_round.append((float((step_ms + serve_ms + deliver_ms).max()), float(bytes_out.max())))
    print(json.dumps(dict(round=rounds, step_ms_max=round(float(step_ms.max()), 3), step_ms_mean=round(float(step_ms.mean()), 3),
                          serve_ms_max=round(float(serve_ms.max()), 3), deliver_ms_max=round(float(deliver_ms.max()), 3),
                          remote_records=[int(x) for x in remote], bytes_out_max=int(bytes_out.max()),
                          active=int(M[:, Wn].sum()) if kad else None)), flush=True)
    if rounds > 5000:
        raise RuntimeError("did not terminate")
torch.cuda.synchronize()
dn = [done_to_numpy(s.finished()) for s in steppers]
d = np.concatenate(dn)
if (not kad or mig) and os.environ.get("OVS_MODEL_CHECK", "1") == "1":
    # every lookup against the single-context route of the same ring (the parity the tests assert)
    from oversim_amd import KbrEngine
    del steppers
    torch.cuda.empty_cache()
    d = d[np.argsort(d["qid"])]
    assert np.array_equal(d["qid"], np.arange(Wn * m))
    with KbrEngine(0) as e:
        e.set_params(params)
        if mig:
            e.kad_load_device(inputs[0]["ids_t"].data_ptr(), inputs[0]["xy_t"].data_ptr(), n)
        else:
            e.chord_load_device(inputs[0]["ids_t"].data_ptr(), inputs[0]["xy_t"].data_ptr(), n)
        kk = torch.cat([I["keys_t"] for I in inputs]); ss = torch.cat([I["src_t"] for I in inputs])
        out = torch.empty((kk.shape[0], 16), dtype=torch.uint8, device=dev)
        rp = torch.empty(kk.shape[0], dtype=torch.int32, device=dev) if mig else None
        e.lookup_device(kk.data_ptr(), ss.data_ptr(), kk.shape[0], out.data_ptr(), torch.cuda.current_stream().cuda_stream,
                        rpcs_ptr=rp.data_ptr() if mig else None)
        torch.cuda.synchronize()
        ref = out.cpu().numpy().reshape(-1).view(np.dtype([("responsible", "<u4"), ("hops", "<u2"), ("status", "u1"),
                                                           ("one_way_hops", "u1"), ("latency_ns", "<i8")]))
    for f in ("responsible", "hops", "status", "one_way_hops", "latency_ns"):
        bad = int((d[f].astype(np.int64) != ref[f].astype(np.int64)).sum())
        assert bad == 0, f"{f}: {bad} lookups differ from the single-context route"
    if mig:
        bad = int((d["pad"].astype(np.int64) != rp.cpu().numpy().astype(np.int64)).sum())
        assert bad == 0, f"rpcs: {bad} lookups differ from the single-context route"
    print(json.dumps(dict(check="sharded == single-context route", lookups=int(len(d)))), flush=True)
# a real node's round: the arcs' kernels, then the records over xGMI -- spread over the 7 links of a
# GPU (all-to-all: each peer gets ~1/7), at --xgmi-gbs per link and direction.  One cohort pays kernel
# + exchange per round; with two cohorts (the native loop's default) one cohort's exchange runs under
# the other's kernel, so a round costs about max(kernel, exchange) + min(kernel, exchange) / 2.
xs = [(k, b / (Wn - 1 if Wn > 1 else 1) / (a.xgmi_gbs * 1e9) * 1e3) for k, b in per_round]
model = dict(exchange_ms=round(sum(x for _, x in xs), 3), one_cohort_ms=round(sum(k + x for k, x in xs), 3),
             two_cohorts_ms=round(sum(max(k, x) + min(k, x) / 2 for k, x in xs), 3), xgmi_gbs_per_link=a.xgmi_gbs)
print(json.dumps(dict(model_per_arc=model)), flush=True)
print(json.dumps(dict(summary=True, workload=a.workload, world=Wn, rounds=rounds, lookups=int(len(d)),
                      ok=int((d["status"] == 0).sum()), mean_hops=float(d["hops"].mean()),
                      step_ms_per_rank=[round(float(x), 3) for x in tot["step_ms"]],
                      serve_ms_per_rank=[round(float(x), 3) for x in tot["serve_ms"]],
                      deliver_ms_per_rank=[round(float(x), 3) for x in tot["deliver_ms"]],
                      bytes_out_per_rank=[int(x) for x in tot["sent"]], wall_s=round(time.time() - t_start, 1))),
      flush=True)
