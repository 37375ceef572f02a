"""CPU tests of the C ABI: the library loads, exports every declared symbol, and the
host-only entry points (parameters, .ini binding) behave like the reference's config."""
from __future__ import annotations

import re
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent


def declared_symbols() -> set[str]:
    syms = set()
    for h in (ROOT / "include").glob("*.h"):
        txt = re.sub(r"/\*.*?\*/", "", h.read_text(), flags=re.S)
        syms |= set(re.findall(r"\b(ovs_[a-z0-9_]+)\s*\(", txt))
    return syms


def test_library_exports_every_declared_symbol():
    import oversim_amd
    L = oversim_amd.lib()
    syms = declared_symbols()
    assert len(syms) >= 15
    for s in sorted(syms):
        assert hasattr(L, s), f"{s} declared in include/ but not exported"
    assert L.ovs_abi_version() == 12


def test_params_default_matches_default_ini():
    from oversim_amd import Params
    p = Params.chord()
    assert (p.keyLength, p.hopCountMax, p.successorListSize, p.numFingerCandidates) == (160, 50, 8, 3)
    assert (p.lookupRedundantNodes, p.lookupParallelRpcs, p.lookupMerge) == (1, 1, 0)
    assert p.rpcUdpTimeout == 1.5 and p.lookupTimeout == 10.0 and p.datarate == 10e6
    k = Params.kademlia()
    assert (k.k, k.s, k.b, k.lookupRedundantNodes, k.lookupParallelRpcs, k.lookupMerge) == (8, 8, 1, 8, 3, 1)
    e = Params.epichord()    # default.ini:145-164
    assert (e.successorListSize, e.cacheTTL, e.lookupRedundantNodes, e.lookupParallelRpcs, e.lookupMerge) == \
        (4, 120.0, 3, 1, 1)


def test_epichord_params_from_ini():
    """**.overlay*.epichord.* keys bind for the EpiChord overlay (EpiChord.ned names)."""
    from oversim_amd import Params
    from oversim_amd.kbr import OVERLAY_EPICHORD
    ini = """
[General]
**.overlay*.epichord.cacheTTL = 60s
**.overlay*.epichord.successorListSize = 6
**.overlay*.chord.successorListSize = 8
"""
    p = Params.from_ini(ini, overlay=OVERLAY_EPICHORD)
    assert (p.successorListSize, p.cacheTTL) == (6, 60.0)


def test_params_from_reference_default_ini_text():
    """The reference's own default.ini lines bind to the same fields (first match wins)."""
    from oversim_amd import OVERLAY_KADEMLIA, Params
    ini = """
[General]
**.overlay*.chord.successorListSize = 8
**.overlay*.chord.extendedFingerTable = false
**.overlay*.kademlia.lookupRedundantNodes = 8
**.overlay*.kademlia.lookupParallelRpcs = 3
**.overlay*.kademlia.lookupMerge = true
**.overlay*.kademlia.k = 8
**.overlay*.*.hopCountMax = 50
**.overlay*.*.keyLength = 160
**.overlay*.*.lookupRedundantNodes = 1
**.overlay*.*.lookupParallelRpcs = 1
**.overlay*.*.lookupMerge = false
**.rpcUdpTimeout = 1.5s
SimpleUnderlayNetwork.overlayTerminal*.udp.jitter = 0.1
**.tier1*.kbrTestApp.testMsgSize = 100B

[Config KadAlpha1]
extends = Base
**.overlay*.kademlia.lookupParallelRpcs = 1

[Config Base]
**.overlay*.*.hopCountMax = 40
SimpleUnderlayNetwork.overlayTerminal*.udp.jitter = 0
**.rpcUdpTimeout = 1500ms
"""
    p = Params.from_ini(ini)
    assert p.successorListSize == 8 and p.lookupRedundantNodes == 1 and p.lookupMerge == 0
    assert p.jitter == 0.1 and p.rpcUdpTimeout == 1.5 and p.testMsgSize == 100
    k = Params.from_ini(ini, "KadAlpha1", overlay=OVERLAY_KADEMLIA)
    assert (k.lookupParallelRpcs, k.lookupRedundantNodes, k.lookupMerge, k.hopCountMax) == (1, 8, 1, 40)
    assert k.jitter == 0.0 and abs(k.rpcUdpTimeout - 1.5) < 1e-15
    c = Params.from_ini(ini, "Base")
    assert c.hopCountMax == 40 and c.lookupParallelRpcs == 1


def test_params_ini_errors():
    from oversim_amd import KbrError, Params
    with pytest.raises(KbrError):
        Params.from_ini("[General]\n**.overlay*.*.hopCountMax = ${10, 20}\n")
    with pytest.raises(KbrError):
        Params.from_ini("[General]\n**.overlay*.chord.routingType = \"hop-by-hop\"\n")
    with pytest.raises(KbrError):
        Params.from_ini("[General]\n**.overlay*.*.recordRoute = true\n")
    with pytest.raises(KbrError):
        Params.from_ini("[General]\n**.overlay*.*.routeMsgAcks = true\n")
    with pytest.raises(KbrError):
        Params.from_ini("[General]\n", "NoSuchConfig")
    with pytest.raises(KbrError):
        Params.from_ini("[General]\n**.rpcUdpTimeout = fast\n")


def test_params_chordlarge_semi_recursive():
    """[Config ChordLarge] (omnetpp.ini:75-85) overrides default.ini's iterative Chord routing."""
    from oversim_amd import Params
    ini = """
[Config ChordLarge]
**.routingType = "semi-recursive"
**.targetOverlayTerminalNum = 10000

[General]
**.overlay*.chord.routingType = "iterative"
**.overlay*.*.recNumRedundantNodes = 3
**.overlay*.*.recordRoute = false
**.overlay*.*.routeMsgAcks = false
"""
    assert Params.from_ini(ini).routingType == 0
    p = Params.from_ini(ini, "ChordLarge")
    assert (p.routingType, p.recNumRedundantNodes) == (1, 3)
    assert Params.from_ini('[General]\n**.routingType = "full-recursive"\n').routingType == 2
    # Kademlia's bucket refresh lookups (Kademlia.cc:1483-1487) run exhaustive-iterative
    assert Params.from_ini('[General]\n**.routingType = "exhaustive-iterative"\n').routingType == 3
    # verify.ini [Config ChordSource]
    assert Params.from_ini('[General]\n**.routingType = "source-routing-recursive"\n').routingType == 4


def test_reference_default_ini_parses():
    """If the reference tree is present (this container only), its default.ini binds cleanly."""
    from oversim_amd import Params
    f = Path("/root/reference/simulations/default.ini")
    if not f.exists():
        pytest.skip("reference not present")
    p = Params.from_ini(f.read_text())
    assert (p.successorListSize, p.hopCountMax, p.keyLength, p.lookupRedundantNodes) == (8, 50, 160, 1)
    assert p.jitter == pytest.approx(0.1) and p.testMsgSize == 100 and p.rpcUdpTimeout == 1.5


def test_workload_ids_sorted_unique():
    from oversim_amd import workload as W
    ids = W.sorted_unique_ids(5000, 3)
    v = [int(sum(int(w[i]) << (32 * i) for i in range(5))) for w in ids]
    assert all(a < b for a, b in zip(v, v[1:]))
    xy = W.coordinates(5000, 3)
    assert xy.shape == (5000, 2) and np.all(np.abs(xy) < 400)
    xy2 = W.coordinates(20000, 3)
    assert np.all(np.abs(xy2) <= 75)


def test_params_kademlia_large():
    """[Config KademliaLarge] (omnetpp.ini:113-126) binds k = 16, lookupRedundantNodes = 16, s = 8,
    alpha = 1 over default.ini (omnetpp.ini ends with `include ./default.ini`: textual inclusion).
    The engine takes these tables (two 96 B blocks per bucket) since round 3."""
    from oversim_amd import OVERLAY_KADEMLIA, Params
    ini = """
[Config KademliaLarge]
**.overlayType = "oversim.overlay.kademlia.KademliaModules"
**.overlay.kademlia.lookupRedundantNodes = 16
**.overlay.kademlia.s = 8
**.overlay.kademlia.k = 16
**.overlay.kademlia.lookupMerge = true
**.overlay.kademlia.lookupParallelPaths = 1
**.overlay.kademlia.lookupParallelRpcs = 1

[General]
**.overlay*.kademlia.lookupParallelRpcs = 3
"""
    p = Params.from_ini(ini, "KademliaLarge", overlay=OVERLAY_KADEMLIA)
    assert (p.k, p.s, p.lookupRedundantNodes, p.lookupParallelRpcs, p.lookupMerge) == (16, 8, 16, 1, 1)
    ref = Path("/root/reference/simulations")
    if (ref / "omnetpp.ini").exists():
        text = (ref / "omnetpp.ini").read_text().replace("include ./default.ini", (ref / "default.ini").read_text())
        q = Params.from_ini(text, "KademliaLarge", overlay=OVERLAY_KADEMLIA)
        assert (q.k, q.s, q.lookupRedundantNodes, q.lookupParallelRpcs) == (16, 8, 16, 1)
        assert q.lookupMerge == 1 and q.hopCountMax == 50
