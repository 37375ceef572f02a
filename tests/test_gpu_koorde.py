"""Koorde on the GPU (K3, oversim_amd/csrc/koorde.hip) against the oracle: the de Bruijn state
the builder derives, Koorde::findNode with KoordeFindNodeExtMessage extensions (fresh, carried
over several responders, and past the key length), whole lookups over parameter variants incl.
hop sequences and FindNodeCall counts, the committed golden vectors, the timed device-pointer
path at 2^20 nodes, and the calls Koorde does not support."""
from __future__ import annotations

from pathlib import Path

import numpy as np
import pytest
import torch

from oversim_amd import KbrEngine, KbrError, Params, workload as W
from oversim_amd.kbr import KOORDE_EXT_DTYPE
from oracle_lib import OracleNet, koorde_params

pytestmark = pytest.mark.gpu
GOLD = Path(__file__).resolve().parent / "golden"
FIELDS = ("responsible", "hops", "status", "one_way_hops", "latency_ns")
NONE = 0xFFFFFFFF
OUT = np.dtype([("responsible", "<u4"), ("hops", "<u2"), ("status", "u1"), ("one_way_hops", "u1"),
                ("latency_ns", "<i8")])
VARIANTS = {"default": {}, "sls8": dict(successorListSize=8), "db8_sb2": dict(deBruijnListSize=8, shiftingBits=2),
            "no_other": dict(useOtherLookup=0), "no_suc": dict(useSucList=0), "sb1": dict(shiftingBits=1),
            "sb8": dict(shiftingBits=8), "small": dict(successorListSize=4, deBruijnListSize=4, shiftingBits=3)}


def _engine_params(**kw):
    return Params.koorde().replace(**kw)


def _load(engine, net, **kw):
    engine.set_params(_engine_params(**kw))
    engine.koorde_load(net.ids, net.xy)


@pytest.mark.parametrize("n", [2, 17, 3000, 1 << 16])
def test_state_matches_oracle(engine: KbrEngine, n):
    net = W.population(n, 11)
    _load(engine, net)
    o = OracleNet("koorde", net.ids, net.xy)
    for a, b in zip(engine.koorde_state(), o.koorde_state()):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("variant", ["default", "db8_sb2", "no_suc", "sb1"])
def test_find_node_chains_match_oracle(engine: KbrEngine, variant):
    kw = VARIANTS[variant]
    n = 5000
    net = W.population(n, 12)
    _load(engine, net, **kw)
    o = OracleNet("koorde", net.ids, net.xy, koorde_params(**kw))
    rng = np.random.default_rng(13)
    m = 2000
    node = rng.integers(0, n, m).astype(np.uint32)
    keys = np.concatenate([W.random_keys(m // 2, rng), net.ids[rng.integers(0, n, m - m // 2)]])
    ext = np.zeros(m, dtype=KOORDE_EXT_DTYPE)
    ext["step"] = 1
    # five responders in a row, each fed the extension the previous response carried
    for _ in range(5):
        nxt, ext_out = engine.koorde_find_node(node, keys, ext)
        for i in range(m):
            h, rk, st = o.koorde_find_node(int(node[i]), keys[i], ext["route_key"][i] if ext["has_route_key"][i] else None,
                                           int(ext["step"][i]))
            assert int(nxt[i]) == (NONE if h is None else h), i
            if h is None:
                continue
            assert int(ext_out["step"][i]) == st and bool(ext_out["has_route_key"][i]) == (rk is not None), i
            if rk is not None:
                assert np.array_equal(ext_out["route_key"][i], rk), i
        ok = nxt != NONE
        node = np.where(ok, nxt, node).astype(np.uint32)
        ext = np.where(ok, ext_out, ext)


def test_find_node_past_the_key_length_throws(engine: KbrEngine):
    net = W.population(2000, 14)
    _load(engine, net)
    o = OracleNet("koorde", net.ids, net.xy)
    rng = np.random.default_rng(15)
    m = 1000
    node = rng.integers(0, 2000, m).astype(np.uint32)
    keys = W.random_keys(m, rng)
    ext = np.zeros(m, dtype=KOORDE_EXT_DTYPE)
    ext["step"] = rng.integers(150, 170, m)
    ext["has_route_key"] = 1
    # half of the route keys just after the node's own key: inside (node, succ0], where the
    # de Bruijn step reads key bits -- past the key length that throws
    rk = net.ids[rng.integers(0, 2000, m)].copy()
    own = net.ids[node].copy()
    own[:, 0] += 1
    half = rng.random(m) < 0.5
    rk[half] = own[half]
    ext["route_key"] = rk
    nxt, _ = engine.koorde_find_node(node, keys, ext)
    for i in range(m):
        h, _, _ = o.koorde_find_node(int(node[i]), keys[i], ext["route_key"][i], int(ext["step"][i]))
        assert int(nxt[i]) == (NONE if h is None else h), i
    assert (nxt == NONE).any()


@pytest.mark.parametrize("variant", list(VARIANTS))
def test_route_matches_oracle(engine: KbrEngine, variant):
    kw = VARIANTS[variant]
    n = 3000
    net = W.population(n, 16)
    _load(engine, net, **kw)
    o = OracleNet("koorde", net.ids, net.xy, koorde_params(**kw))
    k1, s1 = W.lookups(net.ids, 3000, 17, node_ids=True)
    k2, s2 = W.lookups(net.ids, 3000, 18, node_ids=False)
    keys, src = np.concatenate([k1, k2]), np.concatenate([s1, s2])
    g = engine.lookup(keys, src, record_hops=True, count_rpcs=True)
    r = o.route(keys, src, record_hops=True, count_rpcs=True)
    for f in FIELDS + ("rpcs",):
        bad = np.nonzero(g[f].astype(np.int64) != r[f].astype(np.int64))[0]
        assert len(bad) == 0, (f, bad[:8], g[f][bad[:8]], r[f][bad[:8]])
    assert np.array_equal(g["hop_seq"], r["hop_seq"])


@pytest.mark.parametrize("name", ["koorde_n2000", "koorde_n2000_sb2_nosuc"])
def test_route_reproduces_golden(engine: KbrEngine, name):
    g = np.load(GOLD / f"{name}.npz")
    engine.set_params(Params.koorde().replace(
        successorListSize=int(g["successorListSize"]), deBruijnListSize=int(g["deBruijnListSize"]),
        shiftingBits=int(g["shiftingBits"]), useOtherLookup=int(g["useOtherLookup"]), useSucList=int(g["useSucList"])))
    engine.koorde_load(g["ids"], g["xy"])
    r = engine.lookup(g["keys"], g["src"], record_hops=True, count_rpcs=True)
    for f in FIELDS + ("rpcs",):
        assert np.array_equal(r[f].astype(np.int64), g[f].astype(np.int64)), f
    assert np.array_equal(r["hop_seq"][:, :g["hop_seq"].shape[1]], g["hop_seq"])


def test_timed_path_large_ring_vs_oracle(engine: KbrEngine):
    """The device-pointer path bench.py times (OVS_DEVICE_PTRS, no hop recording asked for) on a
    2^20-node ring: a sample against the oracle, the whole batch for its structural property."""
    n, m = 1 << 20, 400_000
    net = W.population(n, 19)
    _load(engine, net)
    dev = torch.device("cuda", 0)
    keys, src = W.lookups(net.ids, m, 20, node_ids=False)
    kt = torch.from_numpy(keys.view(np.int32).copy()).to(dev)
    st = torch.from_numpy(src.view(np.int32).copy()).to(dev)
    dout = torch.empty((m, 16), dtype=torch.uint8, device=dev)
    s = torch.cuda.Stream(device=dev)
    torch.cuda.synchronize()
    engine.lookup_device(kt.data_ptr(), st.data_ptr(), m, dout.data_ptr(), s.cuda_stream)
    s.synchronize()
    out = dout.cpu().numpy().view(OUT).ravel()
    o = OracleNet("koorde", net.ids, net.xy)
    idx = np.random.default_rng(21).choice(m, 3000, replace=False)
    r = o.route(keys[idx], src[idx], record_hops=False)
    for f in FIELDS:
        assert np.array_equal(out[f][idx].astype(np.int64), r[f].astype(np.int64)), f
    ok = out["status"] == 0
    assert ok.mean() > 0.95
    # every delivered lookup ends at the key's responsible node: the first ID >= key, wrapping
    ids = np.array([int.from_bytes(x.astype("<u4").tobytes(), "little") for x in net.ids], dtype=object)
    for i in np.nonzero(ok)[0][:20000]:
        k = int.from_bytes(keys[i].astype("<u4").tobytes(), "little")
        rr = int(out["responsible"][i])
        a, b = ids[rr], ids[rr - 1]
        assert (b < k <= a) if rr else (k > b or k <= a), i


def test_unsupported_calls(engine: KbrEngine):
    net = W.population(500, 22)
    _load(engine, net)
    keys, src = W.lookups(net.ids, 10, 23, node_ids=False)
    with pytest.raises(KbrError):
        engine.lookupCall(keys, src, 1)
    with pytest.raises(KbrError, match="fixed"):
        engine.set_params(Params.koorde().replace(shiftingBits=2))
    engine.set_params(Params.koorde().replace(lookupParallelRpcs=2))
    with pytest.raises(KbrError, match="Koorde"):
        engine.lookup(keys, src)
