"""KBRTestApp statistics.

CPU: the oracle's restatement of KBRTestApp::deliver / evaluateData / finishApp +
GlobalStatistics against hand-counted answers on a crafted batch, and the .sca
writer round trip.  GPU: the engine's reduction (ovs_kbrtest_stats_batch) against
the oracle on real route results -- integer counters bit-exact, fp64 summaries
within 1e-12 relative (the reference's own sums are order dependent: it adds
doubles in event order, the engine in a fixed tree order).
"""
from __future__ import annotations

import math
from pathlib import Path

import numpy as np
import pytest

from oracle_lib import SD_FIELDS, OracleNet, chord_params, kad_params
from oversim_amd import ROUTE_OUT_DTYPE, workload as W

GOLD = Path(__file__).resolve().parent / "golden"
INT_FIELDS = ("num_sent", "num_delivered", "num_dropped", "num_lookup_failed", "hop_count_sum", "latency_sum_ns")


def _crafted():
    g = np.load(GOLD / "chord_n9.npz")
    ids, xy = g["ids"], g["xy"]
    # 8 lookups from 3 sources: OK+match, OK+mismatch (dropped), failed
    src = np.array([0, 0, 0, 1, 1, 2, 2, 2], np.uint32)
    keys = ids[[3, 4, 5, 6, 7, 8, 1, 2]].copy()
    resp = np.array([3, 4, 0, 6, 0xFFFFFFFF, 8, 1, 5], np.uint32)      # #2 and #7 mismatch, #4 failed
    status = np.array([0, 0, 0, 0, 1, 0, 0, 0], np.uint8)
    hops = np.array([2, 3, 1, 4, 0, 2, 5, 1], np.uint8)
    lat = np.array([100_000_000, 250_000_000, 1, 3_000_000_000, -1, 7, 999, 5], np.int64)
    res = {"responsible": resp, "hops": hops.astype(np.uint16), "status": status, "one_way_hops": hops,
           "latency_ns": lat}
    return ids, xy, keys, src, res


def _cstddev(vals):
    n = len(vals)
    if n == 0:
        return {"count": 0, "mean": 0.0, "stddev": 0.0, "min": 0.0, "max": 0.0}
    s = sum(vals)
    sq = sum(v * v for v in vals)
    var = (sq - s * s / n) / (n - 1) if n > 1 else 0.0
    return {"count": n, "mean": s / n, "stddev": math.sqrt(max(var, 0.0)), "min": min(vals), "max": max(vals)}


def test_oracle_stats_hand_counted():
    ids, xy, keys, src, res = _crafted()
    o = OracleNet("chord", ids, xy, chord_params())
    T = 2.0
    st = o.kbrtest_stats(res, keys, src, T, lookupNodeIds=True, testMsgSize=100)
    assert (st["num_sent"], st["num_delivered"], st["num_dropped"], st["num_lookup_failed"]) == (8, 5, 2, 1)
    delivered = [0, 1, 3, 5, 6]
    assert st["hop_count_sum"] == sum(int(res["one_way_hops"][i]) for i in delivered)
    assert st["latency_sum_ns"] == sum(int(res["latency_ns"][i]) for i in delivered)
    assert st["hop_count_mean"] == pytest.approx(st["hop_count_sum"] / 5, rel=1e-15)
    assert st["latency_mean_s"] == pytest.approx(st["latency_sum_ns"] * 1e-9 / 5, rel=1e-12)
    # per node (9 nodes): sent 3,2,3; delivered 2,1,2; dropped 1,0,1
    d = [2, 1, 2] + [0] * 6
    r = [1, 0, 1] + [0] * 6
    s = [3, 2, 3] + [0] * 6
    exp = {
        "delivered_msgs_per_s": _cstddev([x / T for x in d]),
        "delivered_bytes_per_s": _cstddev([x * 100 / T for x in d]),
        "dropped_msgs_per_s": _cstddev([x / T for x in r]),
        "dropped_bytes_per_s": _cstddev([x * 100 / T for x in r]),
        "delivery_ratio": _cstddev([float(np.float32(a) / np.float32(b)) for a, b in zip(d, s) if b > 0]),
    }
    for f in SD_FIELDS:
        for k in ("count", "mean", "stddev", "min", "max"):
            assert st[f][k] == pytest.approx(exp[f][k], rel=1e-12, abs=1e-15), (f, k)
    # lookupNodeIds = false: nothing is dropped, mismatches are delivered
    st2 = o.kbrtest_stats(res, keys, src, T, lookupNodeIds=False)
    assert (st2["num_delivered"], st2["num_dropped"]) == (7, 0)
    # measured lifetime below MIN_MEASURED = 0.1 s: no per-node statistics
    st3 = o.kbrtest_stats(res, keys, src, 0.05)
    assert all(st3[f]["count"] == 0 for f in SD_FIELDS)


def test_sca_round_trip(tmp_path):
    from oversim_amd.kbr import KbrTestStats
    from oversim_amd.stats import read_sca, scalars, write_sca
    st = KbrTestStats()
    st.num_sent, st.num_delivered = 10, 8
    st.hop_count_mean, st.latency_mean_s = 3.25, 0.4321
    st.delivered_msgs_per_s.count, st.delivered_msgs_per_s.mean = 100, 0.0125
    st.delivery_ratio.count, st.delivery_ratio.mean, st.delivery_ratio.stddev = 90, 0.8, 0.1
    p = write_sca(tmp_path / "r.sca", st, sim_time_s=1000.0, config="ChordInet", output_stddev=True)
    sc = read_sca(p)
    assert sc["GlobalStatistics: Simulation Time"] == 1000.0
    assert sc["Vector: KBRTestApp: One-way Hop Count.mean"] == 3.25
    assert sc["Vector: KBRTestApp: One-way Latency.mean"] == 0.4321
    assert sc["KBRTestApp: One-way Delivered Messages/s.mean"] == 0.0125
    assert sc["KBRTestApp: One-way Delivery Ratio.stddev"] == 0.1
    assert "KBRTestApp: One-way Dropped Messages/s.mean" not in sc      # never collected
    names = [n for n, _ in scalars(st, 1.0)]
    assert names[0] == "GlobalStatistics: Simulation Time"
    assert names[1:3] == sorted(names[1:3])                            # std::map order
    text = p.read_text()
    assert text.startswith("version 2\nrun ChordInet-0-")
    assert 'scalar SimpleUnderlayNetwork.globalObserver.globalStatistics \t"KBRTestApp: One-way Delivery Ratio.mean"' in text


# ---------------------------------------------------------------- GPU parity

def _check(gpu, orc):
    for f in INT_FIELDS:
        assert int(getattr(gpu, f)) == int(orc[f]), f
    assert gpu.hop_count_mean == pytest.approx(orc["hop_count_mean"], rel=1e-12)
    assert gpu.latency_mean_s == pytest.approx(orc["latency_mean_s"], rel=1e-12)
    for f in SD_FIELDS:
        g, o = getattr(gpu, f), orc[f]
        assert g.count == o["count"], f
        for k in ("mean", "stddev", "min", "max"):
            assert getattr(g, k) == pytest.approx(o[k], rel=1e-12, abs=1e-12), (f, k)


@pytest.mark.gpu
def test_gpu_stats_crafted(engine):
    from oversim_amd import Params
    ids, xy, keys, src, res = _crafted()
    engine.set_params(Params.chord())
    engine.chord_load(ids, xy)
    o = OracleNet("chord", ids, xy, chord_params())
    for T, nid in ((2.0, True), (2.0, False), (0.05, True), (1e6, True)):
        g = engine.kbrtest_stats(res, keys, src, T, lookupNodeIds=nid)
        _check(g, o.kbrtest_stats(res, keys, src, T, lookupNodeIds=nid))
    g = engine.kbrtest_stats(res, keys, src, 2.0)
    assert list(g.status_count)[:2] == [7, 1]
    hist = np.zeros(64, np.int64)
    for i in (0, 1, 3, 5, 6):
        hist[res["one_way_hops"][i]] += 1
    assert np.array_equal(np.array(list(g.hop_hist)), hist)
    assert (g.hop_count_min, g.hop_count_max) == (2, 5)
    assert (g.latency_min_ns, g.latency_max_ns) == (7, 3_000_000_000)


@pytest.mark.gpu
@pytest.mark.parametrize("node_ids", [True, False])
def test_gpu_stats_chord_routes(engine, node_ids):
    from oversim_amd import Params
    net = W.population(20000, 31)
    keys, src = W.lookups(net.ids, 200_000, 32, node_ids=node_ids)
    # hopCountMax = 4 makes part of the batch fail (HOPMAX) so every branch is exercised
    for hcm in (50, 4):
        engine.set_params(Params.chord().replace(hopCountMax=hcm))
        engine.chord_load(net.ids, net.xy)
        r = engine.lookup(keys, src)
        o = OracleNet("chord", net.ids, net.xy, chord_params(hopCountMax=hcm))
        for T in (600.0, 0.01):
            _check(engine.kbrtest_stats(r, keys, src, T, lookupNodeIds=True),
                   o.kbrtest_stats(r, keys, src, T, lookupNodeIds=True))


@pytest.mark.gpu
def test_gpu_stats_kademlia_routes(engine):
    from oversim_amd import Params
    net = W.population(15000, 41)
    keys, src = W.lookups(net.ids, 100_000, 42, node_ids=True)
    engine.set_params(Params.kademlia().replace(lookupParallelRpcs=1))
    engine.kad_load(net.ids, net.xy)
    r = engine.lookup(keys, src)
    o = OracleNet("kademlia", net.ids, net.xy, kad_params(lookupParallelRpcs=1))
    _check(engine.kbrtest_stats(r, keys, src, 1000.0), o.kbrtest_stats(r, keys, src, 1000.0))


def test_route_out_dtype_matches_abi():
    assert ROUTE_OUT_DTYPE.itemsize == 16


# ---------------------------------------------------------------- lookup test (kbrLookupTest)

def _crafted_lookups():
    """8 LookupResponses from 3 sources: valid + right node, valid + wrong first sibling, invalid."""
    g = np.load(GOLD / "chord_n9.npz")
    ids, xy = g["ids"], g["xy"]
    src = np.array([0, 0, 0, 1, 1, 2, 2, 2], np.uint32)
    keys = ids[[3, 4, 5, 6, 7, 8, 1, 2]].copy()
    first = np.array([3, 4, 0, 6, 0xFFFFFFFF, 8, 1, 5], np.uint32)      # #2 and #7 wrong, #4 invalid
    sib = np.full((8, 3), 0xFFFFFFFF, np.uint32)
    sib[:, 0] = first
    sib[[0, 1, 2, 3, 5, 6, 7], 1] = 7
    nsib = np.where(first == 0xFFFFFFFF, 0, 2).astype(np.uint32)
    valid = (first != 0xFFFFFFFF).astype(np.uint8)
    hops = np.array([2, 3, 1, 4, 6, 2, 5, 1], np.uint16)
    lat = np.array([100_000_000, 250_000_000, 1, 3_000_000_000, -1, 7, 999, 5], np.int64)
    res = {"num_siblings": nsib, "hops": hops, "status": np.where(valid == 1, 0, 3).astype(np.uint8),
           "is_valid": valid, "latency_ns": lat, "siblings": sib}
    return ids, xy, keys, src, res


def test_oracle_lookup_stats_hand_counted():
    ids, xy, keys, src, res = _crafted_lookups()
    o = OracleNet("chord", ids, xy, chord_params())
    st = o.kbrtest_lookup_stats(res, keys, src, 2.0, lookupNodeIds=True, failureLatency=10.0)
    ok = [0, 1, 3, 5, 6]
    assert (st["num_sent"], st["num_success"], st["num_failed"], st["num_invalid"]) == (8, 5, 3, 1)
    assert st["hop_count_sum"] == sum(int(res["hops"][i]) for i in ok)
    assert st["failed_hop_count_sum"] == 1 + 6 + 1
    assert st["success_latency_sum_ns"] == sum(int(res["latency_ns"][i]) for i in ok)
    lat_s = [res["latency_ns"][i] * 1e-9 for i in ok]
    assert st["success_latency_mean_s"] == pytest.approx(sum(lat_s) / 5, rel=1e-12)
    assert st["total_latency_mean_s"] == pytest.approx((sum(lat_s) + 3 * 10.0) / 8, rel=1e-12)
    assert st["failed_hop_count_mean"] == pytest.approx(8 / 3, rel=1e-15)
    per_node_succ = [2, 1, 2] + [0] * 6
    per_node_fail = [1, 1, 1] + [0] * 6
    exp = {"successful_lookups_per_s": _cstddev([v / 2.0 for v in per_node_succ]),
           "failed_lookups_per_s": _cstddev([v / 2.0 for v in per_node_fail]),
           "success_ratio": _cstddev([float(np.float32(2) / np.float32(3)), 0.5, float(np.float32(2) / np.float32(3))])}
    for f in exp:
        for k in ("count", "mean", "stddev", "min", "max"):
            assert st[f][k] == pytest.approx(exp[f][k], rel=1e-12, abs=1e-15), (f, k)
    # lookupNodeIds = false: every valid response counts
    st2 = o.kbrtest_lookup_stats(res, keys, src, 2.0, lookupNodeIds=False)
    assert (st2["num_success"], st2["num_failed"], st2["num_invalid"]) == (7, 1, 1)


def test_sca_lookup_scalars(tmp_path):
    from oversim_amd.kbr import KbrTestLookupStats
    from oversim_amd.stats import read_sca, write_sca
    lk = KbrTestLookupStats()
    lk.num_sent, lk.num_success, lk.num_failed = 10, 9, 1
    lk.hop_count_mean, lk.success_latency_mean_s, lk.total_latency_mean_s = 4.5, 0.25, 1.225
    lk.failed_hop_count_mean = 7.0
    lk.success_ratio.count, lk.success_ratio.mean = 100, 0.9
    sc = read_sca(write_sca(tmp_path / "l.sca", None, 100.0, lookup=lk))
    assert sc["Vector: KBRTestApp: Lookup Hop Count.mean"] == 4.5
    assert sc["Vector: KBRTestApp: Lookup Total Latency.mean"] == 1.225
    assert sc["Vector: KBRTestApp: Failed Lookup Hop Count.mean"] == 7.0
    assert sc["KBRTestApp: Lookup Success Ratio.mean"] == 0.9
    assert "KBRTestApp: Successful Lookups/s.mean" not in sc


LK_INT = ("num_sent", "num_success", "num_failed", "num_invalid", "hop_count_sum", "failed_hop_count_sum",
          "success_latency_sum_ns")


def _check_lookup(gpu, orc):
    from oracle_lib import LOOKUP_SD_FIELDS
    for f in LK_INT:
        assert int(getattr(gpu, f)) == int(orc[f]), f
    for f in ("hop_count_mean", "failed_hop_count_mean", "success_latency_mean_s", "total_latency_mean_s"):
        assert getattr(gpu, f) == pytest.approx(orc[f], rel=1e-12), f
    for f in LOOKUP_SD_FIELDS:
        g, o = getattr(gpu, f), orc[f]
        assert g.count == o["count"], f
        for k in ("mean", "stddev", "min", "max"):
            assert getattr(g, k) == pytest.approx(o[k], rel=1e-12, abs=1e-12), (f, k)


@pytest.mark.gpu
def test_gpu_lookup_stats_crafted(engine):
    from oversim_amd import Params
    ids, xy, keys, src, res = _crafted_lookups()
    engine.set_params(Params.chord())
    engine.chord_load(ids, xy)
    o = OracleNet("chord", ids, xy, chord_params())
    for T, nid in ((2.0, True), (2.0, False), (0.05, True)):
        _check_lookup(engine.kbrtest_lookup_stats(res, keys, src, T, lookupNodeIds=nid),
                      o.kbrtest_lookup_stats(res, keys, src, T, lookupNodeIds=nid))


@pytest.mark.gpu
@pytest.mark.parametrize("overlay", ["chord", "kademlia"])
def test_gpu_lookup_stats_real_lookups(engine, overlay):
    from oversim_amd import Params
    net = W.population(15000, 51)
    keys, src = W.lookups(net.ids, 100_000, 52, node_ids=True)
    hcm = 4 if overlay == "chord" else 3         # part of the batch fails: every branch is exercised
    if overlay == "chord":
        engine.set_params(Params.chord().replace(hopCountMax=hcm))
        engine.chord_load(net.ids, net.xy)
        o = OracleNet("chord", net.ids, net.xy, chord_params(hopCountMax=hcm))
    else:
        engine.set_params(Params.kademlia().replace(hopCountMax=hcm))
        engine.kad_load(net.ids, net.xy)
        o = OracleNet("kademlia", net.ids, net.xy, kad_params(hopCountMax=hcm))
    r = engine.lookupCall(keys, src)
    ref = o.lookup_call(keys, src)
    assert np.array_equal(r["siblings"], ref["siblings"])
    g = engine.kbrtest_lookup_stats(r, keys, src, 500.0)
    _check_lookup(g, o.kbrtest_lookup_stats(r, keys, src, 500.0))
    assert g.num_failed > 0 and g.num_success > 0
