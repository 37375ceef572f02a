"""oversim_amd -- MI355X-native batched KBR lookup routing for OverSim's Chord and Kademlia.

The product is the C-ABI library libovs_kbr.so (include/ovs_kbr.h) built from
the HIP sources in oversim_amd/csrc; this package is its host-side mirror of
the reference's BaseOverlay / AbstractLookup interface (kbr.py) plus workload
generation (workload.py).
"""
from .kbr import (DEVICE_PTRS, LOOKUP_OUT_DTYPE, LOOKUP_STATUS, NONE, OVERLAY_CHORD,  # noqa: F401
                  OVERLAY_KADEMLIA, ROUTE_OUT_DTYPE, KbrEngine, KbrError, Network, Params, key_from_int, key_to_int, keys_array, lib)

__all__ = ["KbrEngine", "KbrError", "Params", "Network", "lib", "keys_array", "key_from_int", "key_to_int",
           "OVERLAY_CHORD", "OVERLAY_KADEMLIA", "ROUTE_OUT_DTYPE", "LOOKUP_OUT_DTYPE", "LOOKUP_STATUS", "NONE", "DEVICE_PTRS"]
