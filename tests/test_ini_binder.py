"""The .ini binder refuses what the engine does not model (ABI 12).

A stock OverSim config that sets a key which would change a route, a response size or a delay
must get OVS_ENOTSUP naming that key -- never a silently different result.  Keys that only
matter where the engine does not go (churn, maintenance timers, statistics) still bind.
measureAuthBlock is modelled (+100 B per RPC response, CommonMessages.msg:45-47, 57, 73).
"""
from __future__ import annotations

from pathlib import Path

import pytest

from oversim_amd import KbrError, Params
from oversim_amd.kbr import OVERLAY_CHORD, OVERLAY_EPICHORD, OVERLAY_KADEMLIA, OVERLAY_KOORDE

REF = Path("/root/reference/simulations")

# (overlay, ini line, substring the refusal must name)
REFUSED = [
    (OVERLAY_CHORD, "**.optimizeTimeouts = true", "optimizeTimeouts"),
    (OVERLAY_KADEMLIA, "**.optimizeTimeouts = true", "optimizeTimeouts"),
    (OVERLAY_CHORD, 'SimpleUnderlayNetwork.overlayTerminal*.udp.delayFaultType = "live_all"', "delayFaultType"),
    (OVERLAY_KADEMLIA, 'SimpleUnderlayNetwork.overlayTerminal*.udp.delayFaultType = "simulation"', "delayFaultType"),
    (OVERLAY_CHORD, 'SimpleUnderlayNetwork.overlayTerminal*.udp.delayFaultType = "live_planetlab"', "delayFaultType"),
    (OVERLAY_CHORD, '**.neighborCache.ncsType = "vivaldi"', "ncsType"),
    (OVERLAY_KADEMLIA, "**.overlay*.kademlia.proximityRouting = true\n**.routingType = \"semi-recursive\"",
     "proximityRouting"),
    (OVERLAY_KADEMLIA, "**.overlay*.kademlia.proximityNeighborSelection = true", "proximityNeighborSelection"),
    (OVERLAY_KADEMLIA, "**.overlay*.kademlia.enableManagedConnections = true", "enableManagedConnections"),
    (OVERLAY_KADEMLIA, "**.overlay*.kademlia.activePing = true", "activePing"),
    (OVERLAY_KADEMLIA, "**.overlay*.kademlia.secureMaintenance = true", "secureMaintenance"),
    (OVERLAY_KADEMLIA, "**.overlay*.kademlia.pingNewSiblings = true", "pingNewSiblings"),
    (OVERLAY_KADEMLIA, "**.overlay*.kademlia.altRecMode = true", "altRecMode"),
    (OVERLAY_CHORD, "**.overlay*.chord.proximityRouting = true\n**.overlay*.chord.extendedFingerTable = true",
     "proximityRouting"),
    (OVERLAY_CHORD, "*.globalObserver.globalNodeList.maliciousNodeProbability = 0.1", "maliciousNodeProbability"),
    (OVERLAY_CHORD, "*.globalObserver.globalNodeList.maliciousNodeChange = true", "maliciousNodeChange"),
    (OVERLAY_CHORD, "network = oversim.underlay.inetunderlay.InetUnderlayNetwork", "network"),
    (OVERLAY_CHORD, "simtime-scale = -12", "simtime-scale"),
    (OVERLAY_CHORD, '**.overlayType = "oversim.overlay.pastry.PastryModules"', "overlayType"),
    (OVERLAY_CHORD, 'SimpleUnderlayNetwork.churnGenerator*.channelTypes = '
                    '"oversim.common.simple_ethernetline oversim.common.simple_dsl"', "channelTypes"),
    (OVERLAY_CHORD, 'SimpleUnderlayNetwork.churnGenerator*.channelTypes = "oversim.common.simple_ethernetline_lossy"',
     "channelTypes"),
    (OVERLAY_CHORD, 'SimpleUnderlayNetwork.churnGenerator*.channelTypesRx = "oversim.common.simple_dsl"',
     "channelTypesRx"),
    (OVERLAY_CHORD, "**.overlay*.*.recordRoute = true", "recordRoute"),
    (OVERLAY_CHORD, "**.overlay*.*.routeMsgAcks = true", "routeMsgAcks"),
    (OVERLAY_CHORD, "network = ${a, b}", "parameter studies"),
]


@pytest.mark.parametrize("overlay,line,key", REFUSED, ids=[f"{k}-{i}" for i, (_, _, k) in enumerate(REFUSED)])
def test_refused_key_is_named(overlay, line, key):
    with pytest.raises(KbrError) as e:
        Params.from_ini(f"[General]\n{line}\n", overlay=overlay)
    assert key in str(e.value), str(e.value)
    assert "ENOTSUP" in str(e.value)


# settings that leave a lookup over the loaded tables unchanged, so they bind
ACCEPTED = [
    (OVERLAY_KADEMLIA, "**.overlay*.kademlia.proximityRouting = true"),   # iterative: findNode serves FindNodeCalls
    (OVERLAY_CHORD, "**.overlay*.chord.proximityRouting = true"),         # only extendedFingerTable's candidates
    (OVERLAY_CHORD, "**.neighborCache.enableNeighborCache = true"),       # no timeouts from it without optimizeTimeouts
    (OVERLAY_CHORD, '**.neighborCache.ncsType = "none"'),
    (OVERLAY_CHORD, '**.neighborCache.ncsType = "vivaldi"\n**.neighborCache.ncsSendBackOwnCoords = false'),
    (OVERLAY_CHORD, 'SimpleUnderlayNetwork.overlayTerminal*.udp.delayFaultType = "no_fault"'),
    (OVERLAY_CHORD, "**.optimizeTimeouts = false"),
    (OVERLAY_CHORD, '*.underlayConfigurator.churnGeneratorTypes = "oversim.common.LifetimeChurn"'),
    (OVERLAY_KADEMLIA, '**.overlayType = "KademliaModules"'),
]


@pytest.mark.parametrize("overlay,line", ACCEPTED)
def test_unmodelled_but_harmless_keys_bind(overlay, line):
    Params.from_ini(f"[General]\n{line}\n", overlay=overlay)


def test_measure_auth_block_binds():
    assert Params.chord().measureAuthBlock == 0
    p = Params.from_ini("[General]\n**.overlay*.*.measureAuthBlock = true\n")
    assert p.measureAuthBlock == 1
    k = Params.from_ini("[Config A]\n**.overlay*.kademlia.measureAuthBlock = true\n[General]\n"
                        "**.overlay*.*.measureAuthBlock = false\n", "A", overlay=OVERLAY_KADEMLIA)
    assert k.measureAuthBlock == 1
    with pytest.raises(KbrError):
        Params.from_ini("[General]\n**.overlay*.*.measureAuthBlock = maybe\n")


def test_channel_types_bind_datarate_and_access_delay():
    p = Params.from_ini('[General]\nSimpleUnderlayNetwork.churnGenerator*.channelTypes = "oversim.common.simple_dsl"\n')
    assert (p.datarate, p.accessDelay) == (1e6, pytest.approx(0.020))
    q = Params.from_ini('[General]\nSimpleUnderlayNetwork.churnGenerator*.channelTypes = '
                        '"oversim.common.simple_ethernetline"\n')
    assert (q.datarate, q.accessDelay) == (10e6, 0.0)
    # the engine's explicit override wins
    r = Params.from_ini('[General]\nSimpleUnderlayNetwork.churnGenerator*.channelTypes = "oversim.common.simple_dsl"\n'
                        'ovs.datarate = 100Mbps\n')
    assert r.datarate == 100e6


def test_overlay_type_must_match():
    with pytest.raises(KbrError, match="bound for kademlia"):
        Params.from_ini('[General]\n**.overlayType = "oversim.overlay.chord.ChordModules"\n', overlay=OVERLAY_KADEMLIA)


def test_ini_file_resolves_include(tmp_path):
    (tmp_path / "base.ini").write_text("[General]\n**.overlay*.*.hopCountMax = 33\n**.overlay*.*.measureAuthBlock = true\n")
    (tmp_path / "run.ini").write_text("[Config X]\n**.overlay*.chord.successorListSize = 4\n\ninclude ./base.ini\n")
    p = Params.from_ini_file(tmp_path / "run.ini", "X")
    assert (p.hopCountMax, p.successorListSize, p.measureAuthBlock) == (33, 4, 1)
    with pytest.raises(KbrError, match="cannot open"):
        Params.from_ini_file(tmp_path / "missing.ini")


# every Chord-family / Kademlia [Config] of the reference's omnetpp.ini (with its default.ini):
# None = binds, else the key the refusal names
OMNETPP = {
    ("Chord", OVERLAY_CHORD): None, ("ChordSimpleSemi", OVERLAY_CHORD): None,
    ("ChordFastStab", OVERLAY_CHORD): None, ("ChordLarge", OVERLAY_CHORD): None,
    ("ChordBroadcast", OVERLAY_CHORD): None,        # its ${...} study is over lifetimeMean (churn), not read
    ("ChordDht", OVERLAY_CHORD): None, ("ChordDhtTrace", OVERLAY_CHORD): None,
    ("ChordInet", OVERLAY_CHORD): "network", ("ChordInet6", OVERLAY_CHORD): "network",
    ("ChordReaSE", OVERLAY_CHORD): "network",
    ("Kademlia", OVERLAY_KADEMLIA): None, ("KademliaLarge", OVERLAY_KADEMLIA): None,
    ("Koorde", OVERLAY_KOORDE): None, ("KoordeLarge", OVERLAY_KOORDE): None,
    ("EpiChord", OVERLAY_EPICHORD): None, ("EpiChordLarge", OVERLAY_EPICHORD): None,
}


@pytest.mark.skipif(not (REF / "omnetpp.ini").exists(), reason="reference not present (GPU box)")
@pytest.mark.parametrize("cfg,overlay", list(OMNETPP))
def test_reference_omnetpp_configs_bind_or_refuse(cfg, overlay):
    want = OMNETPP[(cfg, overlay)]
    if want is None:
        p = Params.from_ini_file(REF / "omnetpp.ini", cfg, overlay=overlay)
        assert p.keyLength == 160 and p.measureAuthBlock == 0 and p.jitter == pytest.approx(0.1)
    else:
        with pytest.raises(KbrError) as e:
            Params.from_ini_file(REF / "omnetpp.ini", cfg, overlay=overlay)
        assert want in str(e.value)


@pytest.mark.skipif(not (REF / "default.ini").exists(), reason="reference not present (GPU box)")
def test_reference_default_and_other_ini_files():
    assert Params.from_ini_file(REF / "default.ini").successorListSize == 8
    # maidsafe.ini [Config Kademlia] turns on managed connections (maidsafe.ini:5-47)
    with pytest.raises(KbrError, match="enableManagedConnections"):
        Params.from_ini_file(REF / "maidsafe.ini", "Kademlia", overlay=OVERLAY_KADEMLIA)
    # verify.ini: the short module names bind; KademliaInet is another underlay
    assert Params.from_ini_file(REF / "verify.ini", "ChordSource").routingType == 4
    Params.from_ini_file(REF / "verify.ini", "Kademlia", overlay=OVERLAY_KADEMLIA)
    with pytest.raises(KbrError, match="network"):
        Params.from_ini_file(REF / "verify.ini", "KademliaInet", overlay=OVERLAY_KADEMLIA)
    # validation.ini runs EpiChord; thesis.ini's network / overlayType studies are refused
    Params.from_ini_file(REF / "validation.ini", "lookup-1way", overlay=OVERLAY_EPICHORD)
    with pytest.raises(KbrError, match="parameter studies"):
        Params.from_ini_file(REF / "thesis.ini", "TestInetSimpleKbr")
