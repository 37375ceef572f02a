"""Kademlia maintenance-round fixtures shared by the CPU and GPU tests: a partially joined network
(the converged tables of most nodes, a few joiners that know one bootstrap node each) as explicit
tables, built with the oracle's snapshot rule and routingAdd (test infrastructure only)."""
from __future__ import annotations

import numpy as np

from oracle_lib import OracleNet, kad_params


def partial_join(ids, xy, frac: float, seed: int, params=None):
    """(tables dict for orc_kad_build_tables / ovs_kad_load_tables, joiner indices).  Members hold
    the snapshot tables of the member-only network; each joiner pinged a random member
    (Kademlia::joinOverlay, Kademlia.cc:270-303): the member's handleRpcCall routingAdd()s the
    joiner, the joiner's PingResponse routingAdd()s the member (1328-1420)."""
    params = params or kad_params()
    n = len(ids)
    rng = np.random.default_rng(seed)
    join = np.sort(rng.choice(n, size=max(1, int(n * frac)), replace=False)).astype(np.uint32)
    mem = np.setdiff1d(np.arange(n, dtype=np.uint32), join)
    sub = OracleNet("kademlia", ids[mem], xy[mem], params)
    ssib, scnt, snodes = sub.kad_tables()
    S5, k = 5 * params.s, params.k
    sib = np.full((n, S5), 0xFFFFFFFF, np.uint32)
    cnt = np.zeros((n, 160), np.uint8)
    nodes = np.full((n, 160, k), 0xFFFFFFFF, np.uint32)
    remap = np.concatenate([mem, np.array([0xFFFFFFFF], np.uint32)])
    sib[mem] = remap[np.where(ssib == 0xFFFFFFFF, len(mem), ssib)]
    cnt[mem] = scnt
    nodes[mem] = remap[np.where(snodes == 0xFFFFFFFF, len(mem), snodes)]
    net = OracleNet("kademlia", ids, xy, params, tables=dict(siblings=sib, bucket_count=cnt, bucket_nodes=nodes))
    boot = mem[rng.integers(0, len(mem), size=len(join))]
    for j, b in zip(join, boot):
        net.routing_add(int(b), int(j), True)     # the bootstrap answers the joiner's PingCall
        net.routing_add(int(j), int(b), True)     # the joiner gets the PingResponse
    s2, c2, n2 = net.kad_tables()
    return dict(siblings=s2, bucket_count=c2, bucket_nodes=n2), join
