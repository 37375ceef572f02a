"""The drop-in boundary from C: tests/c_consumer/route_batch (gcc, include/ovs_kbr.h, linked to
libovs_kbr.so; built by __graft_entry__.build()) binds the reference's own .ini parameter names,
loads a network, routes a KBRTestApp one-way batch and a LookupCall batch -- no Python or torch in
the process -- and its outputs must equal the oracle's."""
from __future__ import annotations

import struct
import subprocess
from pathlib import Path

import numpy as np
import pytest

from oversim_amd import kbr, workload as W
from oracle_lib import OracleNet, chord_params, kad_params

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parent.parent
EXE = ROOT / "tests" / "c_consumer" / "route_batch"

INI = {
    kbr.OVERLAY_CHORD: "[General]\n**.overlay*.chord.successorListSize = 8\n",
    kbr.OVERLAY_KADEMLIA: "[General]\n**.overlay*.kademlia.lookupParallelRpcs = 3\n**.overlay*.kademlia.k = 8\n",
}


def _run(tmp_path, overlay, ids, xy, keys, src, ini):
    fin, fout = tmp_path / "in.bin", tmp_path / "out.bin"
    b = ini.encode()
    with open(fin, "wb") as f:
        f.write(struct.pack("<IQQ", overlay, len(ids), len(keys)))
        for a in (ids.astype("<u4"), xy.astype("<f8"), keys.astype("<u4"), src.astype("<u4")):
            f.write(np.ascontiguousarray(a).tobytes())
        f.write(struct.pack("<I", len(b)) + b)
    subprocess.run([str(EXE), str(fin), str(fout)], check=True, timeout=120)
    raw = fout.read_bytes()
    m = len(keys)
    out = np.frombuffer(raw, dtype=kbr.ROUTE_OUT_DTYPE, count=m)
    off = out.nbytes
    rpcs = np.frombuffer(raw, dtype="<u4", count=m, offset=off)
    off += rpcs.nbytes
    lo = np.frombuffer(raw, dtype=kbr.LOOKUP_OUT_DTYPE, count=m, offset=off)
    off += lo.nbytes
    sib = np.frombuffer(raw, dtype="<u4", offset=off).reshape(m, -1)
    return out, rpcs, lo, sib


@pytest.mark.parametrize("overlay", [kbr.OVERLAY_CHORD, kbr.OVERLAY_KADEMLIA])
def test_c_consumer_matches_oracle(tmp_path, overlay):
    assert EXE.exists(), "tests/c_consumer/route_batch missing: run __graft_entry__.build()"
    net = W.population(3000, 0xC0 + overlay)
    keys, src = W.lookups(net.ids, 4000, 0xC1 + overlay, node_ids=overlay == kbr.OVERLAY_KADEMLIA)
    out, rpcs, lo, sib = _run(tmp_path, overlay, net.ids, net.xy, keys, src, INI[overlay])
    if overlay == kbr.OVERLAY_CHORD:
        o = OracleNet("chord", net.ids, net.xy, chord_params())
    else:
        o = OracleNet("kademlia", net.ids, net.xy, kad_params(lookupParallelRpcs=3))
    e = o.route(keys, src, record_hops=False, count_rpcs=True)
    for f in ("responsible", "hops", "status", "one_way_hops", "latency_ns"):
        assert np.array_equal(out[f], e[f]), f
    assert np.array_equal(rpcs, e["rpcs"])
    c = o.lookup_call(keys, src, -1)
    for f in ("num_siblings", "hops", "status", "is_valid", "latency_ns"):
        assert np.array_equal(lo[f], c[f]), f
    assert np.array_equal(sib, c["siblings"])


EXE2 = ROOT / "tests" / "c_consumer" / "sharded_route"


@pytest.mark.parametrize("overlay,world,top", [(kbr.OVERLAY_CHORD, 3, 6), (kbr.OVERLAY_CHORD, 4, 0),
                                               (kbr.OVERLAY_KADEMLIA, 3, 0), (kbr.OVERLAY_KADEMLIA, 3, 3)])
def test_c_consumer_sharded_route(tmp_path, overlay, world, top):
    """The multi-GPU route from C: tests/c_consumer/sharded_route runs W ranks as
    pthreads, one context per arc, over the library's in-process exchange through
    ovs_shard_route_batch / ovs_kad_shard_route_batch -- the round loop in C++ behind the ABI -- and
    its results equal ovs_route_batch on the whole network and the oracle."""
    assert EXE2.exists(), "tests/c_consumer/sharded_route missing: run __graft_entry__.build()"
    net = W.population(20000, 0xC5 + overlay + world)
    keys, src = W.lookups(net.ids, 6000, 0xC6 + overlay, node_ids=(world % 2 == 1))
    fin, fout = tmp_path / "in.bin", tmp_path / "out.bin"
    with open(fin, "wb") as f:
        f.write(struct.pack("<IQQ", overlay, len(net.ids), len(keys)))
        for a in (net.ids.astype("<u4"), net.xy.astype("<f8"), keys.astype("<u4"), src.astype("<u4")):
            f.write(np.ascontiguousarray(a).tobytes())
        f.write(struct.pack("<Ii", world, top))
    subprocess.run([str(EXE2), str(fin), str(fout)], check=True, timeout=300)
    raw = fout.read_bytes()
    m = len(keys)
    sh = np.frombuffer(raw, dtype=kbr.ROUTE_OUT_DTYPE, count=m)
    off = sh.nbytes
    rpcs = np.frombuffer(raw, dtype="<u4", count=m, offset=off)
    off += rpcs.nbytes
    ref = np.frombuffer(raw, dtype=kbr.ROUTE_OUT_DTYPE, count=m, offset=off)
    rounds = struct.unpack_from("<I", raw, off + ref.nbytes)[0]
    assert rounds >= 2
    for f in ("responsible", "hops", "status", "one_way_hops", "latency_ns"):
        assert np.array_equal(sh[f], ref[f]), f
    if overlay == kbr.OVERLAY_CHORD:
        e = OracleNet("chord", net.ids, net.xy, chord_params()).route(keys, src, record_hops=False)
    else:
        e = OracleNet("kademlia", net.ids, net.xy, kad_params(lookupParallelRpcs=3)).route(keys, src, record_hops=False,
                                                                                          count_rpcs=True)
        assert np.array_equal(rpcs, e["rpcs"])
    for f in ("responsible", "hops", "status", "one_way_hops", "latency_ns"):
        assert np.array_equal(sh[f], e[f]), f
