"""Parity of the exact paths bench.py times, on the exact inputs it times them on.

bench.py routes device-resident batches with `KbrEngine.lookup_device` (OVS_DEVICE_PTRS, no hop
recording, on a non-default stream): that is the `k_chord_lanes<REC=0, RECORD=0, SHARD=0>` and
`k_kad_route<A, RECORD=0, EX, LK=0>` instantiations, which the record-hops tests elsewhere do not
run.  Each test builds the bench workload (oversim_amd.workload.bench_inputs), routes the full
batch through lookup_device and checks
  * a sample against the CPU oracle (bit-exact: responsible node, hops, status, one-way hops,
    int64-ns latency, and the FindNodeCall count for Kademlia) -- lazy oracle tables at the
    2^26-node (D) and 2^24-node (E) sizes, where stored tables would not fit in host memory;
  * size-independent properties over the whole batch.
"""
from __future__ import annotations

import numpy as np
import pytest
import torch

from oversim_amd import KbrEngine, Params, workload as W
from oracle_lib import OracleNet, chord_params, kad_params

pytestmark = pytest.mark.gpu
FIELDS = ("responsible", "hops", "status", "one_way_hops", "latency_ns")
OUT = np.dtype([("responsible", "<u4"), ("hops", "<u2"), ("status", "u1"), ("one_way_hops", "u1"),
                ("latency_ns", "<i8")])


def _route_device(eng: KbrEngine, I: dict, rpcs: bool):
    dev = I["keys_t"].device
    m = I["m"]
    dout = torch.empty((m, 16), dtype=torch.uint8, device=dev)
    drpc = torch.empty(m, dtype=torch.int32, device=dev) if rpcs else None
    s = torch.cuda.Stream(device=dev)
    torch.cuda.synchronize()
    eng.lookup_device(I["keys_t"].data_ptr(), I["src_t"].data_ptr(), m, dout.data_ptr(), s.cuda_stream,
                      rpcs_ptr=drpc.data_ptr() if rpcs else None)
    s.synchronize()
    out = dout.cpu().numpy().view(OUT).ravel()
    return out, (drpc.cpu().numpy().view(np.uint32) if rpcs else None)


def _host_inputs(I: dict):
    if I["ids"] is not None:
        return I["ids"], I["xy"], I["keys"], I["src"]
    return (I["ids_t"].cpu().numpy().view(np.uint32), I["xy_t"].cpu().numpy(),
            I["keys_t"].cpu().numpy().view(np.uint32), I["src_t"].cpu().numpy().view(np.uint32))


def _check_sample(out, rpcs, ref, idx, label):
    for f in FIELDS:
        a = out[f][idx].astype(np.int64)
        b = np.asarray(ref[f]).astype(np.int64)
        bad = np.nonzero(a != b)[0]
        assert len(bad) == 0, f"{label}: {f} differs at sample {idx[bad[:6]]}: gpu {a[bad[:6]]} oracle {b[bad[:6]]}"
    if rpcs is not None:
        assert np.array_equal(rpcs[idx].astype(np.int64), ref["rpcs"].astype(np.int64)), f"{label}: rpcs differ"


def _top64(w):
    return (w[:, 4].astype(np.uint64) << np.uint64(32)) | w[:, 3].astype(np.uint64)


def _chord_properties(out, ids, keys, src, label):
    assert np.all(out["status"] == 0), f"{label}: failed lookups {np.bincount(out['status'])}"
    # the responsible node of a key is its ring successor (Chord::isSiblingFor, Chord.cc:452-457);
    # decided on the top 64 bits wherever they are unambiguous
    top, ktop = _top64(ids), _top64(keys)
    pos = np.searchsorted(top, ktop, side="left")
    clear = (pos == len(top)) | (top[np.minimum(pos, len(top) - 1)] != ktop)
    expect = np.where(pos == len(top), 0, pos)
    assert np.array_equal(out["responsible"][clear], expect[clear].astype(np.uint32)), label
    # KBRTestApp one-way hop count: + 1 for the route message unless the source is responsible
    assert np.array_equal(out["one_way_hops"].astype(np.int64),
                          out["hops"].astype(np.int64) + (out["responsible"] != src)), label
    # every counted hop costs at least the 4 serialisation delays (83 B call + 87 B response)
    assert np.all(out["latency_ns"] >= out["hops"].astype(np.int64) * 272000), label


def _xor_closest(top, ktop):
    """Index of the XOR-closest node to each key on the top 64 bits: a descent of the binary trie
    over the sorted ids, taking the key's bit where some node continues the prefix."""
    lo = np.zeros(len(ktop), dtype=np.int64)
    hi = np.full(len(ktop), len(top), dtype=np.int64)
    prefix = np.zeros(len(ktop), dtype=np.uint64)
    for b in range(63, -1, -1):
        bit = np.uint64(1) << np.uint64(b)
        split = np.clip(np.searchsorted(top, prefix | bit, side="left"), lo, hi)
        want = ((ktop >> np.uint64(b)) & np.uint64(1)).astype(bool)
        nlo, nhi = np.where(want, split, lo), np.where(want, hi, split)
        go = nlo < nhi
        lo, hi = np.where(go, nlo, np.where(want, lo, split)), np.where(go, nhi, np.where(want, split, hi))
        prefix |= np.where(go == want, bit, np.uint64(0))
    return lo, hi - lo


def _kad_properties(out, ids, keys, label):
    assert np.all(out["status"] == 0), f"{label}: failed lookups {np.bincount(out['status'])}"
    # the result is the XOR-closest node to the key (isSiblingFor(c, K, 1) holds only there: every
    # closer node would lie inside c's sibling radius, Kademlia.cc:888-962); checked on a sample
    # wherever the top 64 bits decide it
    idx = np.arange(0, len(out), 13)[:300_000]
    best, nbest = _xor_closest(_top64(ids), _top64(keys[idx]))
    clear = nbest == 1
    assert clear.mean() > 0.99
    assert np.array_equal(out["responsible"][idx][clear], best[clear].astype(np.uint32)), label


@pytest.mark.timeout(300)
def test_timed_path_config_a():
    """Config A: Chord 1000 nodes on nodes_2d_15000.xml coordinates, 100k node-ID
    lookups, seed 0x4213 -- the whole batch against the oracle."""
    dev = torch.device("cuda", 0)
    I = W.bench_inputs("A", dev)
    assert I["seed"] == 0x4213 and I["n_total"] == 1000 and I["m"] == 100_000
    with KbrEngine(0) as eng:
        eng.set_params(Params.chord())
        eng.chord_load_device(I["ids_t"].data_ptr(), I["xy_t"].data_ptr(), I["n_total"])
        out, _ = _route_device(eng, I, rpcs=False)
    ids, xy, keys, src = _host_inputs(I)
    assert np.all(out["status"] == 0)
    assert np.array_equal(ids[out["responsible"]], keys)     # node-ID keys end at the key's node
    idx = np.arange(I["m"])
    ref = OracleNet("chord", ids, xy).route(keys, src, record_hops=False)
    _check_sample(out, None, ref, idx, "A")


@pytest.mark.timeout(600)
def test_timed_path_config_c():
    """Config C (the default bench line): 2^20-node ring, the full 10M-lookup batch."""
    dev = torch.device("cuda", 0)
    I = W.bench_inputs("C", dev)
    with KbrEngine(0) as eng:
        eng.set_params(Params.chord())
        eng.chord_load_device(I["ids_t"].data_ptr(), I["xy_t"].data_ptr(), I["n_total"])
        out, _ = _route_device(eng, I, rpcs=False)
    ids, xy, keys, src = _host_inputs(I)
    _chord_properties(out, ids, keys, src, "C")
    idx = np.arange(0, I["m"], 37)[:200_000]
    ref = OracleNet("chord", ids, xy, lazy=True).route(keys[idx], src[idx], record_hops=False)
    _check_sample(out, None, ref, idx, "C")


@pytest.mark.timeout(900)
def test_timed_path_config_d():
    """Config D on one GPU: 2^26-node ring (122 GB of tables), the full 8M-lookup batch; 100k-lookup
    oracle sample over lazy tables."""
    dev = torch.device("cuda", 0)
    I = W.bench_inputs("D", dev)
    with KbrEngine(0) as eng:
        eng.set_params(Params.chord())
        eng.chord_load_device(I["ids_t"].data_ptr(), I["xy_t"].data_ptr(), I["n_total"])
        out, _ = _route_device(eng, I, rpcs=False)
    ids, xy, keys, src = _host_inputs(I)
    del I
    torch.cuda.empty_cache()
    _chord_properties(out, ids, keys, src, "D")
    idx = np.arange(0, len(out), 79)[:100_000]
    ref = OracleNet("chord", ids, xy, lazy=True).route(keys[idx], src[idx], record_hops=False)
    _check_sample(out, None, ref, idx, "D")


@pytest.mark.timeout(600)
def test_timed_path_config_b():
    """Config B: Kademlia 15 000 nodes, alpha = 1, the full 1M node-ID lookup batch with RPC counts."""
    dev = torch.device("cuda", 0)
    I = W.bench_inputs("B", dev)
    with KbrEngine(0) as eng:
        eng.set_params(Params.kademlia().replace(lookupParallelRpcs=1))
        eng.kad_load_device(I["ids_t"].data_ptr(), I["xy_t"].data_ptr(), I["n_total"])
        out, rpcs = _route_device(eng, I, rpcs=True)
    ids, xy, keys, src = _host_inputs(I)
    assert np.all(out["status"] == 0)
    # node-ID keys: the lookup ends at the key's node
    R = out["responsible"]
    assert np.array_equal(ids[R], keys)
    idx = np.arange(0, I["m"], 5)[:200_000]
    ref = OracleNet("kademlia", ids, xy, kad_params(lookupParallelRpcs=1)).route(keys[idx], src[idx],
                                                                                 record_hops=False, count_rpcs=True)
    _check_sample(out, rpcs, ref, idx, "B")


@pytest.mark.timeout(900)
def test_timed_path_config_e():
    """Config E on one GPU: Kademlia 2^24 nodes, alpha = 3, the full 4M random-key batch with RPC
    counts; 50k-lookup oracle sample over lazy tables."""
    dev = torch.device("cuda", 0)
    I = W.bench_inputs("E", dev)
    with KbrEngine(0) as eng:
        eng.set_params(Params.kademlia().replace(lookupParallelRpcs=3))
        eng.kad_load_device(I["ids_t"].data_ptr(), I["xy_t"].data_ptr(), I["n_total"])
        out, rpcs = _route_device(eng, I, rpcs=True)
    ids, xy, keys, src = _host_inputs(I)
    del I
    torch.cuda.empty_cache()
    _kad_properties(out, ids, keys, "E")
    idx = np.arange(0, len(out), 61)[:50_000]
    ref = OracleNet("kademlia", ids, xy, kad_params(lookupParallelRpcs=3), lazy=True).route(
        keys[idx], src[idx], record_hops=False, count_rpcs=True)
    _check_sample(out, rpcs, ref, idx, "E")
