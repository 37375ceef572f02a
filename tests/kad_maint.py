"""Kademlia maintenance-round fixtures shared by the CPU and GPU tests: a partially joined network
(the converged tables of most nodes, a few joiners that know one bootstrap node each) as explicit
tables, built with the oracle's snapshot rule and routingAdd (test infrastructure only)."""
from __future__ import annotations

import numpy as np

from oracle_lib import OracleNet, kad_params

NONE = 0xFFFFFFFF


def partial_join(ids, xy, frac: float, seed: int, params=None, csr: bool = False):
    """(tables dict for orc_kad_build_tables(_csr) / ovs_kad_load_tables(_csr), joiner indices).
    Members hold the snapshot tables of the member-only network; each joiner pinged a random member
    (Kademlia::joinOverlay, Kademlia.cc:270-303): the member's handleRpcCall routingAdd()s the
    joiner, the joiner's PingResponse routingAdd()s the member (1328-1420).  csr: the tables in CSR
    form (any b / bucket size); else k-stride arrays (b = 1, bucketType kademlia)."""
    params = params or kad_params()
    n = len(ids)
    rng = np.random.default_rng(seed)
    join = np.sort(rng.choice(n, size=max(1, int(n * frac)), replace=False)).astype(np.uint32)
    mem = np.setdiff1d(np.arange(n, dtype=np.uint32), join)
    # nkademlia has no snapshot rule (its buckets depend on the arrival order): members start from
    # the kademlia snapshot of the member network, which nkademlia's routingAdd then extends
    sp = params.replace(bucketType=0) if params.bucketType == 1 else params
    sub = OracleNet("kademlia", ids[mem], xy[mem], sp)
    remap = np.concatenate([mem, np.array([NONE], np.uint32)])
    S5 = 5 * params.s
    sib = np.full((n, S5), NONE, np.uint32)
    ssib, soff, snodes = sub.kad_tables_csr()
    sib[mem] = remap[np.where(ssib == NONE, len(mem), ssib)]
    NB = sub.num_buckets()
    cnt = np.zeros((n, NB), np.int64)
    cnt[mem] = np.diff(soff).reshape(len(mem), NB)
    off = np.concatenate([[0], np.cumsum(cnt.reshape(-1))]).astype(np.uint64)
    nodes = np.empty(int(off[-1]), np.uint32)
    mo = np.repeat(np.arange(n), NB)      # row -> node
    # member rows in member order keep their order inside the full-network CSR
    src_rows = np.zeros(n * NB, np.int64) - 1
    src_rows.reshape(n, NB)[mem] = np.arange(len(mem) * NB).reshape(len(mem), NB)
    for r in np.nonzero(cnt.reshape(-1))[0]:
        q = src_rows[r]
        nodes[off[r]:off[r + 1]] = remap[snodes[soff[q]:soff[q + 1]]]
    del mo
    net = OracleNet("kademlia", ids, xy, params, tables=dict(siblings=sib, bucket_off=off, bucket_nodes=nodes))
    boot = mem[rng.integers(0, len(mem), size=len(join))]
    for j, b in zip(join, boot):
        net.routing_add(int(b), int(j), True)     # the bootstrap answers the joiner's PingCall
        net.routing_add(int(j), int(b), True)     # the joiner gets the PingResponse
    if csr:
        s2, o2, n2 = net.kad_tables_csr()
        return dict(siblings=s2, bucket_off=o2, bucket_nodes=n2), join
    s2, c2, n2 = net.kad_tables()
    return dict(siblings=s2, bucket_count=c2, bucket_nodes=n2), join
